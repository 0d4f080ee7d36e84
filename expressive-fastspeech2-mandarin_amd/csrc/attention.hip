// Self-attention with a key-padding mask for the FFT blocks, CDNA4 MFMA (bf16 or exact f32).
//
// Reference: transformer/Modules.py:14-25 (bmm(q, k^T) / temperature, masked_fill(mask, -inf),
// softmax(dim=2), bmm(attn, v)) with the head split/merge of transformer/SubLayers.py:36-52.
// The reference materialises the [H*B, T, T] score tensor (94.7 MB fp32 per decoder layer at
// B=64, T=430); here one workgroup owns 64 query rows of one (sequence, head), keeps its Q
// fragments in registers, streams 64-key K/V tiles through LDS only up to the sequence's key
// length (padded keys beyond it are never touched) and keeps an online softmax in f32.
//
// Per 64-key tile, wave w (16 query rows):
//   S = Q K^T      4 key blocks x (128/32) bf16 MFMAs (or 128/16 x 4 f32 MFMAs)
//   online max / sum across the 16 lanes that share a row (xor shuffles), O *= exp2(m_old-m_new)
//   P -> LDS (wave-private rows), read back as A fragments
//   O += P V       V is staged TRANSPOSED in LDS (Vt[d][key]) so B fragments are 16-byte reads.
// LDS rows are XOR-swizzled by row so every fragment read is bank-conflict free.
#include <cstdlib>
#include <type_traits>

#include "fs2_common.h"

#ifndef ATTN_ABL
#define ATTN_ABL 0  // analysis builds only (tools/attn_abl.py): bit 0 no exp / max, 1 no QK MFMAs,
#endif              // 2 no PV MFMAs, 3 no K / V DMA wait, 4 no K / V DMA
#ifndef ATTN_TRACE
#define ATTN_TRACE 0  // analysis builds only: per-workgroup shader-clock stamps of attn32_kernel
#endif

#if ATTN_TRACE
__device__ unsigned long long g_attn_stamps[4096 * 8];
extern "C" int fs2_attn_trace_read(void *dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps)) == hipSuccess ? 0 : 1;
}
#endif

namespace {

constexpr int DK = 128;
constexpr int QT = 64;  // query rows per workgroup
constexpr int KT = 64;  // keys per tile

template <int CT>
struct ATraits;
template <>
struct ATraits<FS2_BF16> {
  using T = bf16;
};
template <>
struct ATraits<FS2_F32> {
  using T = float;
  static constexpr int CEp = 4;
};

template <int CT>
__global__ __launch_bounds__(256, 2) void attn_kernel(const typename ATraits<CT>::T *__restrict__ qkv, int64_t qs,
                                                      const int64_t *__restrict__ lens, int T, int H, float scale_log2,
                                                      typename ATraits<CT>::T *__restrict__ out, int64_t os,
                                                      const int32_t *__restrict__ cu, float *__restrict__ lse) {
  using TE = typename ATraits<CT>::T;
  constexpr int ES = sizeof(TE);
  constexpr int CEp = ATraits<CT>::CEp;
  constexpr int KROW = DK * ES;          // bytes per K row (16 or 32 chunks)
  constexpr int VROW = KT * ES;          // bytes per Vt / P row (8 or 16 chunks)
  constexpr int VSW = VROW / 16 - 1;     // swizzle mask for Vt / P rows (7 or 15)
  __shared__ __attribute__((aligned(16))) char Ks[KT * KROW];
  __shared__ __attribute__((aligned(16))) char Vts[DK * VROW];
  __shared__ __attribute__((aligned(16))) char Ps[4 * 16 * VROW];

  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * QT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // padded rows: sequence b is rows b*T.., all T query rows computed, keys >= lens[b] masked;
  // packed rows (cu): sequence b is rows cu[b] .. cu[b+1]-1 and only those exist
  int len;
  int64_t row0;
  if (cu != nullptr) {
    row0 = cu[b];
    len = cu[b + 1] - cu[b];
    T = len;
  } else {
    const int64_t len64 = lens[b];
    len = (int)(len64 < 0 ? 0 : (len64 > T ? T : len64));
    row0 = (int64_t)b * T;
  }
  if (q0 >= T) return;
  const TE *base = qkv + row0 * qs;

  auto koff = [](int row, int chunk) { return row * KROW + ((chunk ^ (row & 15)) << 4); };
  auto voff = [](int row, int chunk) { return row * VROW + ((chunk ^ (row & VSW)) << 4); };

  // ---- Q fragments (registers, whole head dim) -----------------------------------------------
  const int qrow = q0 + 16 * w + (lane & 15);
  const bool q_ok = qrow < T;
  constexpr int QSTEPS = (CT == FS2_BF16) ? DK / 32 : DK / 16;
  using QFrag = typename std::conditional<CT == FS2_BF16, bf16x8, f32x4>::type;
  QFrag qf[QSTEPS];
#pragma unroll
  for (int s = 0; s < QSTEPS; ++s) {
    const int k = (s * 4 + (lane >> 4)) * CEp;
    if (q_ok)
      qf[s] = *reinterpret_cast<const QFrag *>(base + (int64_t)qrow * qs + h * DK + k);
    else
      qf[s] = QFrag{};
  }

  f32x4 oacc[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m_run[j] = -INFINITY;
    l_run[j] = 0.f;
  }

  const int ntiles = (len + KT - 1) / KT;
  char *Pw = Ps + w * 16 * VROW;
  for (int kt = 0; kt < ntiles; ++kt) {
    const int k0 = kt * KT;
    __syncthreads();  // previous tile's K / Vt reads are done
    // K tile: KT rows x KROW bytes
    constexpr int KCH = KT * KROW / 16;
    for (int e = tid; e < KCH; e += 256) {
      const int r = e / (KROW / 16), c = e % (KROW / 16);
      const int key = k0 + r;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (key < T) v = *reinterpret_cast<const uint4 *>(base + (int64_t)key * qs + (H + h) * DK + c * CEp);
      *reinterpret_cast<uint4 *>(Ks + koff(r, c)) = v;
    }
    // V tile transposed: unit = (key pair, 16-byte d chunk)
    constexpr int VUNITS = (KT / 2) * (DK / CEp);
    for (int e = tid; e < VUNITS; e += 256) {
      const int kp = e / (DK / CEp), dc = e % (DK / CEp);
      const int key = k0 + 2 * kp;
      TE v0[CEp], v1[CEp];
      uint4 r0 = make_uint4(0u, 0u, 0u, 0u), r1 = r0;
      const TE *vp = base + (2 * H + h) * DK + dc * CEp;
      if (key < T) r0 = *reinterpret_cast<const uint4 *>(vp + (int64_t)key * qs);
      if (key + 1 < T) r1 = *reinterpret_cast<const uint4 *>(vp + (int64_t)(key + 1) * qs);
      __builtin_memcpy(v0, &r0, 16);
      __builtin_memcpy(v1, &r1, 16);
      const int kk = 2 * kp;  // key within tile (even)
#pragma unroll
      for (int q = 0; q < CEp; ++q) {
        const int d = dc * CEp + q;
        char *dst = Vts + voff(d, kk / CEp) + (kk % CEp) * ES;
        if constexpr (CT == FS2_BF16) {
          bf16 pair[2] = {v0[q], v1[q]};
          uint32_t u;
          __builtin_memcpy(&u, pair, 4);
          *reinterpret_cast<uint32_t *>(dst) = u;
        } else {
          *reinterpret_cast<float2 *>(dst) = make_float2(v0[q], v1[q]);
        }
      }
    }
    __syncthreads();

    // ---- S = Q K^T --------------------------------------------------------------------------
    f32x4 sacc[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < QSTEPS; ++s) {
      const int ch = s * 4 + (lane >> 4);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const QFrag kf = *reinterpret_cast<const QFrag *>(Ks + koff(ni * 16 + (lane & 15), ch));
        if constexpr (CT == FS2_BF16) {
          sacc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], kf, sacc[ni], 0, 0, 0);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) sacc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[s][j], kf[j], sacc[ni], 0, 0, 0);
        }
      }
    }

    // ---- online softmax (rows 4*(lane>>4)+j of the wave's 16, keys ni*16 + (lane&15)) -------
    float alpha[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mx = -INFINITY;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int key = k0 + ni * 16 + (lane & 15);
        float sv = sacc[ni][j] * scale_log2;
        sv = key < len ? sv : -INFINITY;
        sacc[ni][j] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float m_new = fmaxf(m_run[j], mx);
      alpha[j] = exp2f(m_run[j] - m_new);
      m_run[j] = m_new;
      float sum = 0.f;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float p = exp2f(sacc[ni][j] - m_new);
        sacc[ni][j] = p;
        sum += p;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
      l_run[j] = l_run[j] * alpha[j] + sum;
    }
#pragma unroll
    for (int ni = 0; ni < DK / 16; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) oacc[ni][j] *= alpha[j];

    // ---- P -> LDS (wave-private 16 x 64) ---------------------------------------------------
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 4 * (lane >> 4) + j;
        const int key = ni * 16 + (lane & 15);
        *reinterpret_cast<TE *>(Pw + voff(row, key / CEp) + (key % CEp) * ES) = (TE)sacc[ni][j];
      }
    __syncthreads();

    // ---- O += P V -----------------------------------------------------------------------------
    constexpr int PSTEPS = (CT == FS2_BF16) ? KT / 32 : KT / 16;
#pragma unroll
    for (int s = 0; s < PSTEPS; ++s) {
      const int ch = s * 4 + (lane >> 4);
      const QFrag pa = *reinterpret_cast<const QFrag *>(Pw + voff(lane & 15, ch));
#pragma unroll
      for (int ni = 0; ni < DK / 16; ++ni) {
        const QFrag vf = *reinterpret_cast<const QFrag *>(Vts + voff(ni * 16 + (lane & 15), ch));
        if constexpr (CT == FS2_BF16) {
          oacc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vf, oacc[ni], 0, 0, 0);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) oacc[ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j], vf[j], oacc[ni], 0, 0, 0);
        }
      }
    }
  }

  // ---- normalise and store ---------------------------------------------------------------------
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + 16 * w + 4 * (lane >> 4) + j;
    if (q >= T) continue;
    const float inv = l_run[j] > 0.f ? 1.0f / l_run[j] : 0.f;
    TE *orow = out + (row0 + q) * os + h * DK + (lane & 15);
#pragma unroll
    for (int ni = 0; ni < DK / 16; ++ni) orow[ni * 16] = (TE)(oacc[ni][j] * inv);
    // log2-domain log-sum-exp of the scaled scores (the backward's softmax statistics)
    if (lse != nullptr && (lane & 15) == 0)
      lse[(row0 + q) * H + h] = l_run[j] > 0.f ? m_run[j] + __log2f(l_run[j]) : INFINITY;
  }
}


// ------------------------------------------------------------------------------------------------
// bf16 fast path. Same math, different data flow:
//   S^T = K Q^T   (A = K rows from LDS, B = Q fragments in registers): the accumulator holds,
//                 per lane, 16 scores of ONE query (column l&15) -> the softmax row statistics
//                 are per lane, reduced across the 4 lanes of that query with 2 xor-shuffles.
//   O^T = V^T P^T (A = V^T from LDS with ds_read_b64_tr_b16 on the row-major V tile, B = P
//                 straight from the S^T registers): no P round trip through LDS, no transposing
//                 V writes. The k order inside each 32-key MFMA step is permuted identically on
//                 both operands (lane group g takes keys 4g..4g+3 and 16+4g..16+4g+3).
// K and V tiles arrive by LDS-DMA (buffer_load ... lds, OOB rows -> zeros) into a dual-use XOR
// image (row reads and transposed reads conflict-light), double buffered. Workgroups of one
// (utterance, head) are placed on one XCD so its K/V stay in that XCD's L2.
// 16-byte chunk swizzle of K / V row `row` (256 B rows = all 64 banks). The K fragment reads take
// one chunk of 16 consecutive rows: f must be a bijection on rows 16i..16i+15. The transposed V
// reads (ds_read_b64_tr_b16) take, per 32 lanes, one 32-byte chunk PAIR {2m, 2m+1} of 8 consecutive
// rows: f >> 1 must be a bijection on rows 8i..8i+7. f = ((row & 7) << 1) | ((row >> 3) & 1) meets
// both; the round-1 f = ((row & 3) << 2) | ((row >> 2) & 3) gave rows r and r+4 the same pair
// (2-way conflicts on every V read: 2.7 M conflict cycles per decoder attention call, rocprofv3).
__device__ __forceinline__ int kv_swz(int row) { return ((row & 7) << 1) | ((row >> 3) & 1); }
__device__ __forceinline__ int kv_off(int row, int chunk) { return row * 256 + ((chunk ^ kv_swz(row)) << 4); }

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// scores are never NaN (masked keys are -inf): max without NaN canonicalisation. (Inline-asm
// v_max3_f32 here read MFMA results with no wait states -- the hazard recognizer does not see into
// asm -- and took stale accumulator values: a timing-dependent wrong row max.)
__device__ __forceinline__ float max_nn(float a, float b) { return __builtin_fmaxf(a, b); }
// reductions over the 4 lanes of one query (lane groups g = lane >> 4) with the gfx950 row-swap
// permutes: v_permlane16_swap pairs rows (0, 1) / (2, 3), v_permlane32_swap the two halves. No LDS
// round trip (ds_bpermute + lgkmcnt(0), which also waited for the in-flight K / V reads).
__device__ __forceinline__ float rows_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s1 = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float rows_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s1 = max_nn(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
  return max_nn(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

template <int N>
__device__ __forceinline__ void attn_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NWV waves (16 queries each) per workgroup, an NST-deep K/V ring: the DMA of key tile kt+NST-1
// is issued right after the barrier that retires tile kt-1, so each tile has NST-1 tiles of
// compute to land; one counted vmcnt + one barrier per tile.
template <int NWV, int NST, int KTT = KT>
__global__ __launch_bounds__(64 * NWV, 1) void attn_bf16_kernel(const bf16 *__restrict__ qkv, int64_t qs,
                                                                uint32_t qkv_bytes, const int64_t *__restrict__ lens,
                                                                int B, int T, int H, int nqt, float scale_log2,
                                                                bf16 *__restrict__ out, int64_t os,
                                                                const int32_t *__restrict__ cu,
                                                                float *__restrict__ lse) {
  constexpr int QTW = 16 * NWV;          // queries per workgroup
  static_assert(KTT == 64 || KTT == 32, "keys per tile");
  constexpr int PPW = KTT / 4 / NWV;     // K (and V) 1 KiB pieces per wave per tile
  constexpr int LPS = 2 * PPW;           // LDS-DMA loads per wave per tile
  constexpr int STG = 2 * KTT * 256;     // K + V bytes of one tile
  __shared__ __attribute__((aligned(16))) char smem[NST * STG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;

  const int nwg = gridDim.x, id = blockIdx.x;
  const int q8 = nwg >> 3, rem = nwg & 7, xcd = id & 7;
  const int t = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + (id >> 3);
  const int qt = t % nqt, bh = t / nqt, h = bh % H, b = bh / H;
  const int q0 = qt * QTW;
  int len;
  uint32_t seq_base;
  if (cu != nullptr) {  // packed rows: only the sequence's own rows exist
    seq_base = (uint32_t)cu[b];
    len = cu[b + 1] - cu[b];
    T = len;
  } else {
    const int64_t len64 = lens[b];
    len = (int)(len64 < 0 ? 0 : (len64 > T ? T : len64));
    seq_base = (uint32_t)b * (uint32_t)T;
  }
  if (q0 >= T) return;
  const bool active = q0 + 16 * w < T;  // wave-uniform: this wave has queries (else DMA + barriers only)

  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16 *>(qkv), (short)0, (int)qkv_bytes, 0x00020000);
  const uint32_t row_bytes = (uint32_t)qs * 2u;

  // Q^T fragments (B operand): query q0 + 16w + li, head dims 32s + 8g .. +7
  const int qrow = q0 + 16 * w + li;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint32_t off = qrow < T ? (seq_base + qrow) * row_bytes + (uint32_t)(h * DK + 32 * s + 8 * g) * 2u : 0x80000000u;
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    qf[s] = *reinterpret_cast<bf16x8 *>(&v);
  }

  // LDS-DMA of one 64-key tile: 16 pieces of 4 rows x 256 B for K, 16 for V; PPW of each per wave.
  const int prow = lane >> 4, pch = lane & 15;
  auto dma = [&](int k0, int buf) {
    char *Kb = smem + buf * STG;
    char *Vb = Kb + KTT * 256;
#pragma unroll
    for (int it = 0; it < PPW; ++it) {
      const int p = w + NWV * it;
      const int r = 4 * p + prow;
      const int lc = pch ^ kv_swz(r);
      const int key = k0 + r;
      const uint32_t base = key < T ? (seq_base + key) * row_bytes + (uint32_t)lc * 16u : 0x80000000u;
      const uint32_t koff = base == 0x80000000u ? base : base + (uint32_t)((H + h) * DK) * 2u;
      const uint32_t voff = base == 0x80000000u ? base : base + (uint32_t)((2 * H + h) * DK) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(Kb + p * 1024), 16, koff,
                                               0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(Vb + p * 1024), 16, voff,
                                               0, 0, 0);
    }
  };

  f32x4 oacc[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // running max kept in RAW score units (scale > 0 commutes with max): p = exp2(fma(s, c, -m*c))
  float m_run = -INFINITY, l_run = 0.f;

  const int ntiles = (len + KTT - 1) / KTT;
  // the Q loads are waited for with the first tile (they were issued first)
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < ntiles) dma(st * KTT, st);
  // transposed-read lane roles: lane 4q+p of its 16-lane group addresses row q, columns 4p..4p+3.
  // kv_off's swizzle depends on row & 15 only, so rows +16 / +32 are +4 / +8 KiB:
  // only the 8 column-block offsets of row r0 are lane-specific (hoisted out of the key loop).
  const int tq = li >> 2, tp = li & 3;
  int voff[DK / 16];
#pragma unroll
  for (int nd = 0; nd < DK / 16; ++nd) voff[nd] = kv_off(4 * g + tq, nd * 2 + (tp >> 1)) + (tp & 1) * 8;
  // one key tile; MASKED (the last tile only) sets the scores of keys >= len to -inf
  auto tile = [&](int kt, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
    const int k0 = kt * KTT;
    // tile kt landed (this wave's pieces); tiles issued after it may stay in flight
    const int ahead = ntiles - 1 - kt;
    if (NST >= 3 && ahead >= NST - 2)
      attn_vm_wait<LPS * (NST - 2)>();
    else if (NST >= 4 && ahead == 1)
      attn_vm_wait<LPS>();
    else
      attn_vm_wait<0>();
    // tile kt visible to all waves; the buffer of tile kt-1 is free. Raw barrier: __syncthreads()
    // would drain vmcnt to 0 and with it the tiles still in flight.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < ntiles) dma(k0 + (NST - 1) * KTT, (kt + NST - 1) % NST);
    if (!active) return;
    const char *Kb = smem + (kt % NST) * STG;
    const char *Vb = Kb + KTT * 256;

    constexpr int NB = KTT / 16;  // 16-key blocks per tile
    f32x4 sacc[NB];
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
      sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(Kb + kv_off(ni * 16 + li, 4 * s + g));
        sacc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sacc[ni], 0, 0, 0);
      }
    }
    // scores of query li: keys k0 + ni*16 + 4g + j
    if constexpr (MASKED) {
      const int lim = len - k0 - 4 * g;
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ni * 16 + j >= lim) sacc[ni][j] = -INFINITY;
    }
    float mx = m_run;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
      mx = max_nn(max_nn(mx, sacc[ni][0]), sacc[ni][1]);
      mx = max_nn(max_nn(mx, sacc[ni][2]), sacc[ni][3]);
    }
    const float m_new = rows_max(mx);  // includes m_run
    // rescale only when some query's running max moved (alpha == 1 exactly for the others): after
    // the first tiles of a sequence the max rarely moves, and the O rescale is 32 VALU per wave
    if (__builtin_amdgcn_ballot_w64(m_new != m_run) != 0) {
      // raw v_exp_f32 (exp2; underflow -> 0, -inf -> 0): libm exp2f's range reduction is dead work here
      const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * scale_log2);
      l_run *= alpha;
      // scalar multiplies: packed f32 VALU beside MFMAs costs more issue cycles than two scalar
      // ops (cdna_hip_programming.md, VALU issue costs); same products, same bits
#pragma unroll
      for (int nd = 0; nd < DK / 16; ++nd)
#pragma unroll
        for (int q = 0; q < 4; ++q) oacc[nd][q] = __builtin_fmaf(oacc[nd][q], alpha, 0.0f);
    }
    m_run = m_new;
    // p = exp2(s * c - m * c), two running sums (x / y elements, as the packed form summed them)
    const float mc = -m_new * scale_log2;
    float sx = 0.f, sy = 0.f;
    bf16x8 pf[NB / 2];
#pragma unroll
    for (int ni = 0; ni < NB; ++ni)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const float px = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp], scale_log2, mc));
        const float py = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp + 1], scale_log2, mc));
        sx += px;
        sy += py;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp] = (bf16)px;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp + 1] = (bf16)py;
      }
    l_run += rows_sum(sx + sy);

    // V^T fragments 4 at a time ahead of their MFMAs (one read / wait / MFMA chain per fragment
    // left every MFMA waiting out an LDS round trip)
    auto vread = [&](int s2, int nd) {
      const char *vp = Vb + voff[nd] + s2 * 32 * 256;
      auto lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)vp);
      auto hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(vp + 16 * 256));
      bf16x8 vf;
      __builtin_memcpy(&vf, &lo, 8);
      __builtin_memcpy(reinterpret_cast<char *>(&vf) + 8, &hi, 8);
      return vf;
    };
#pragma unroll
    for (int s2 = 0; s2 < NB / 2; ++s2) {
      // this lane's address row r0 = 32*s2 + 4g + tq (block 1), r0 + 16 for block 2
#pragma unroll
      for (int h4 = 0; h4 < DK / 64; ++h4) {
        bf16x8 vf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) vf[i] = vread(s2, 4 * h4 + i);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          oacc[4 * h4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[i], pf[s2], oacc[4 * h4 + i], 0, 0, 0);
      }
    }
  };
  // every tile but the last is fully inside the sequence (keys < len): no masking work there
  for (int kt = 0; kt + 1 < ntiles; ++kt) tile(kt, std::false_type{});
  if (ntiles > 0) tile(ntiles - 1, std::true_type{});

  // O^T[d = nd*16 + 4g + j][query li]
  const int q = q0 + 16 * w + li;
  if (q < T) {
    const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
    if (lse != nullptr && g == 0)  // log2-domain log-sum-exp (m_run is in unscaled score units here)
      lse[((int64_t)seq_base + q) * H + h] = l_run > 0.f ? m_run * scale_log2 + __log2f(l_run) : INFINITY;
    bf16 *orow = out + ((int64_t)seq_base + q) * os + h * DK + 4 * g;
#pragma unroll
    for (int nd = 0; nd < DK / 16; ++nd) {
      bf16x4 o = {(bf16)(oacc[nd][0] * inv), (bf16)(oacc[nd][1] * inv), (bf16)(oacc[nd][2] * inv),
                  (bf16)(oacc[nd][3] * inv)};
      *reinterpret_cast<bf16x4 *>(orow + nd * 16) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 32 queries per wave on v_mfma_f32_32x32x16_bf16 (the decoder's long sequences). Swapped product
// S^T = K Q^T: a lane owns ONE query (column lane & 31) and 16 keys of each 32-key block in its
// registers (rows crow(r, h) = (r & 3) + 8 (r >> 2) + 4 h, h = lane >> 5), so the row max / sum is
// in-lane plus one permlane32 swap. The exponentiated scores are already the B operand of
// O^T = V^T P^T (k-step s = registers 8 (s & 1) .. +7 of block s >> 1, keys in crow order), and
// V^T's A fragments take the same key order from two transposed reads (rows 4h .. 4h+3 and
// 8+4h .. 8+4h+3 of the 16-key step). Each K / V fragment read from LDS feeds a 32-query MFMA:
// half the LDS bytes per FLOP of the 16-query form (whose K and V reads alone were 512 KB per
// 64-key tile per CU at 16 waves). O^T stays in registers: lane = query, so the online-softmax
// rescale is lane-local. K / V tiles: the same LDS-DMA ring as attn_bf16_kernel, rows swizzled
// with the 256-byte-row XOR map under which the b128 row reads and the transposed reads of the
// 32x32x16 operands are both conflict-free (cdna_hip_programming.md, T11 image (b)).
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int kv32_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int kv32_off(int row, int chunk) { return row * 256 + ((chunk ^ kv32_swz(row)) << 4); }

__device__ __forceinline__ rsrc_t make_rsrc_any(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

// Key-split form (SPL; packed rows with their work list, no lse). A sequence longer than
// kSplitKeys keys is cut into kSplitKeys-key ranges, one workgroup per (query tile, head, range):
// each stores its unnormalised O, running max and sum (write-through) in a workspace slot and the
// last range of the (query tile, head) to arrive (an arrival counter) merges them in range order
// and stores the output; a sequence of <= kSplitKeys keys runs exactly the unsplit arithmetic. The
// workgroups take the items of a compact list (attn_items_kernel, once per packed layout: a dense
// (query tile, head, sequence, range) grid over a free-running batch is ~90 % empty workgroups,
// each paying a memory round trip to find out), so the grid is one workgroup per item. A
// sequence's split depends on its own length only: the result does not depend on T.
constexpr int kSplitKeys = 256;
constexpr int kSplitMax = 8;   // ranges per sequence (T <= 2048)
constexpr int kPartLane = 68;  // floats per lane: O^T 64, m, l, 2 pad (17 pieces of 16 bytes)

struct SplitArgs {
  const int *items;  // (b << 16) | (qt << 8) | (s << 4) | h
  const int *count;  // number of items
  float *part;       // partials: slot (tile, head) x kSplitMax ranges x 17 pieces x 256 lanes x 16 B
  int *cnt;          // arrival counters per slot (zero between launches)
};

template <int NWV, int NST, bool SPL = false>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void attn32_kernel(const bf16 *__restrict__ qkv, int64_t qs, uint32_t qkv_bytes,
                                                             const int64_t *__restrict__ lens, int B, int T, int H, int nqt,
                                                             float scale_log2, bf16 *__restrict__ out, int64_t os,
                                                             const int32_t *__restrict__ cu, float *__restrict__ lse,
                                                             int oflags, SplitArgs sa = SplitArgs{}) {
  constexpr int KTT = 64;
  constexpr int QTW = 32 * NWV;       // queries per workgroup
  constexpr int PPW = KTT / 4 / NWV;  // K (and V) 1 KiB pieces per wave per tile
  constexpr int LPS = 2 * PPW;        // LDS-DMA loads per wave per tile
  constexpr int STG = 2 * KTT * 256;  // K + V bytes of one tile
  static_assert(PPW >= 1 && KTT % (4 * NWV) == 0, "pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[NST * STG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;

  // XCD-contiguous work order, as attn_bf16_kernel
  const int nwg = gridDim.x, id = blockIdx.x;
  int qt, h, b, s = 0;
  if constexpr (SPL) {
    // item groups of 4 (consecutive ranges / query tiles of one sequence and head: shared K / V in
    // one L2) dealt round-robin over the XCDs, so a list shorter than the grid still covers all 8
    const int k = id >> 3, t = ((k >> 2) << 5) + ((id & 7) << 2) + (k & 3);
    if (t >= *sa.count) return;
    const int it = sa.items[t];
    b = it >> 16, qt = (it >> 8) & 0xff, s = (it >> 4) & 0xf, h = it & 0xf;
  } else {
    const int q8 = nwg >> 3, rem = nwg & 7, xcd = id & 7;
    const int t = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + (id >> 3);
    qt = t % nqt;
    const int bh = t / nqt;
    h = bh % H, b = bh / H;
  }
  const int q0 = qt * QTW;
  const int T_all = T;
  int len;
  uint32_t seq_base;
  if (cu != nullptr) {
    seq_base = (uint32_t)cu[b];
    len = cu[b + 1] - cu[b];
    T = len;
  } else {
    const int64_t len64 = lens[b];
    len = (int)(len64 < 0 ? 0 : (len64 > T ? T : len64));
    seq_base = (uint32_t)b * (uint32_t)T;
  }
  if (q0 >= T) return;
  int k_lo = 0, k_hi = len, nsp = 1;
  if constexpr (SPL) {
    nsp = (len + kSplitKeys - 1) / kSplitKeys;
    k_lo = s * kSplitKeys;
    k_hi = k_lo + kSplitKeys < len ? k_lo + kSplitKeys : len;
  }
  const bool active = q0 + 32 * w < T;  // wave-uniform
#if ATTN_TRACE
  unsigned long long tst[4];
  tst[0] = __builtin_readcyclecounter();
#endif

  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16 *>(qkv), (short)0, (int)qkv_bytes, 0x00020000);
  const uint32_t row_bytes = (uint32_t)qs * 2u;

  // Q^T fragments (B operand of 32x32x16): query q0 + 32w + r32, head dims 16s + 8hh .. +7
  const int qrow = q0 + 32 * w + r32;
  bf16x8 qf[DK / 16];
#pragma unroll
  for (int s = 0; s < DK / 16; ++s) {
    const uint32_t off = qrow < T ? (seq_base + qrow) * row_bytes + (uint32_t)(h * DK + 16 * s + 8 * hh) * 2u : 0x80000000u;
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    qf[s] = *reinterpret_cast<bf16x8 *>(&v);
  }

  // K / V tile DMA: piece p = w + NWV it is key rows 4p .. 4p + 3 (lane: row 4p + (lane >> 4), 16-byte
  // chunk lane & 15 under the row swizzle). The per-lane part of each piece's source offset is
  // fixed (dbase); a tile adds k0 rows through the scalar offset, and a key past the sequence gets
  // an out-of-range offset (the buffer load returns zeros: V rows of masked keys must be finite)
  const int prow = lane >> 4, pch = lane & 15;
  uint32_t dbase[PPW];
#pragma unroll
  for (int it = 0; it < PPW; ++it) {
    const int r = 4 * (w + NWV * it) + prow;
    dbase[it] = (seq_base + (uint32_t)r) * row_bytes + (uint32_t)(pch ^ kv32_swz(r)) * 16u + (uint32_t)((H + h) * DK) * 2u;
  }
  const uint32_t v_minus_k = (uint32_t)(H * DK) * 2u;  // V columns sit H * DK after K's
  auto dma = [&](int k0, int buf) __attribute__((always_inline)) {
    char *Kb = smem + buf * STG;
    char *Vb = Kb + KTT * 256;
    const int lim = T - k0;
    const uint32_t so = (uint32_t)k0 * row_bytes;
    if (ATTN_ABL & 16) return;
#pragma unroll
    for (int it = 0; it < PPW; ++it) {
      const int p = w + NWV * it;
      const uint32_t vo = 4 * p + prow < lim ? dbase[it] : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(Kb + p * 1024), 16, vo, so,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(Vb + p * 1024), 16, vo,
                                               so + v_minus_k, 0, 0);
    }
  };

  f32x16 oacc[DK / 32];
#pragma unroll
  for (int i = 0; i < DK / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;  // m: raw score units, both lane halves equal; l: this half's keys

  const int ntiles = (k_hi - k_lo + KTT - 1) / KTT;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < ntiles) dma(k_lo + st * KTT, st);
  // transposed V reads: 16-lane group gq = lane >> 4 takes dims 16 (gq & 1) .. +15 of a 32-dim
  // block and key rows 4 (gq >> 1) + q (+ 8 for the second read); lane 4q + p of the group
  // addresses row q, dims 4p .. 4p + 3 (chunk 2 (gq & 1) + (p >> 1), byte 8 (p & 1))
  const int gq = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int vrow = 4 * (gq >> 1) + tq;
  // per-lane LDS offsets of every fragment read, computed once: the row swizzle depends on row & 15
  // only, so a K read is koff[s] + 8 KiB kb and a V read voff[db][half] + 4 KiB s, and with the
  // ring slot a template constant each read is one VGPR + an immediate offset (the per-read
  // address arithmetic was 46 of the ~270 VALU per tile and wave)
  int koff[DK / 16], voff[DK / 32][2];
#pragma unroll
  for (int s = 0; s < DK / 16; ++s) koff[s] = r32 * 256 + (((2 * s + hh) ^ kv32_swz(r32)) << 4);
#pragma unroll
  for (int db = 0; db < DK / 32; ++db) {
    const int ch = 4 * db + 2 * (gq & 1) + (tp >> 1);
    voff[db][0] = kv32_off(vrow, ch) + 8 * (tp & 1);
    voff[db][1] = kv32_off(8 + vrow, ch) + 8 * (tp & 1);
  }
  // online softmax with a lazy running max (FlashAttention-4's threshold): the running reference
  // m_run moves (and O / l are rescaled) only when some lane's tile maximum exceeds it by more than
  // 2^kLazy in the exponentiated domain; otherwise p = exp2((s - m_run) * scale) stays <= 2^kLazy,
  // well inside bf16 / f32 range. The result is the same softmax (O / l and lse are taken against
  // the same reference); the 64-element O rescale no longer runs on nearly every tile.
  constexpr float kLazy = 8.0f;
  auto tile = [&](int kt, auto slot_tag, auto masked_tag) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_tag)::value;
    constexpr bool MASKED = decltype(masked_tag)::value;
    const int k0 = k_lo + kt * KTT;
    const int ahead = ntiles - 1 - kt;
    if (ATTN_ABL & 8)
      ;
    else if (NST >= 3 && ahead >= NST - 2)
      attn_vm_wait<LPS * (NST - 2)>();
    else
      attn_vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < ntiles) dma(k0 + (NST - 1) * KTT, (kt + NST - 1) % NST);
    if (!active) return;
    const char *Kb = smem + SLOT * STG;
    const char *Vb = Kb + KTT * 256;

    // S^T[key][query] for the tile's two 32-key blocks, interleaved: the K fragments of step s + 1
    // are read while the two MFMAs of step s run (64 cycles of matrix work cover each read)
    f32x16 sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb][r] = 0.f;
    bf16x8 kf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) kf[0][kb] = *reinterpret_cast<const bf16x8 *>(Kb + kb * 32 * 256 + koff[0]);
#pragma unroll
    for (int s = 0; s < DK / 16; ++s) {
      if (s + 1 < DK / 16) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          kf[(s + 1) & 1][kb] = *reinterpret_cast<const bf16x8 *>(Kb + kb * 32 * 256 + koff[s + 1]);
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        if (!(ATTN_ABL & 2)) sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s & 1][kb], qf[s], sacc[kb], 0, 0, 0);
    }
    if (ATTN_ABL & 2)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[kb][r] += (float)kf[1][kb][r & 7];
    if constexpr (MASKED) {  // keys >= len -> -inf
      const int lim = len - k0 - 4 * hh;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kb * 32 + (r & 3) + 8 * (r >> 2) >= lim) sacc[kb][r] = -INFINITY;
    }
    if (ATTN_ABL & 1) {  // ablation: P = bf16(S), no max / exp
      bf16x8 pf[KTT / 16];
#pragma unroll
      for (int s = 0; s < KTT / 16; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[s][j] = (bf16)sacc[s >> 1][8 * (s & 1) + j];
#pragma unroll
      for (int s = 0; s < KTT / 16; ++s) {
        bf16x8 vf[DK / 32];
#pragma unroll
        for (int db = 0; db < DK / 32; ++db) {
          auto lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(Vb + s * 16 * 256 + voff[db][0]));
          auto hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(Vb + s * 16 * 256 + voff[db][1]));
          __builtin_memcpy(&vf[db], &lo, 8);
          __builtin_memcpy(reinterpret_cast<char *>(&vf[db]) + 8, &hi, 8);
        }
#pragma unroll
        for (int db = 0; db < DK / 32; ++db)
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[db], pf[s], oacc[db], 0, 0, 0);
      }
      l_run = 1.f;
      return;
    }
    float mx = m_run;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = max_nn(max_nn(mx, sacc[kb][r]), sacc[kb][r + 1]);
    {
      auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = max_nn(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    // first tile: m_run = -inf, so the difference is +inf and every lane takes its maximum
    if (__builtin_amdgcn_ballot_w64((mx - m_run) * scale_log2 > kLazy) != 0) {
      const float alpha = __builtin_amdgcn_exp2f((m_run - mx) * scale_log2);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < DK / 32; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] = __builtin_fmaf(oacc[i][r], alpha, 0.0f);
      m_run = mx;
    }
    const float mc = -m_run * scale_log2;
    float sx = 0.f, sy = 0.f;
    bf16x8 pf[KTT / 16];
#pragma unroll
    for (int s = 0; s < KTT / 16; ++s)
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float px = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[s >> 1][8 * (s & 1) + j], scale_log2, mc));
        const float py = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[s >> 1][8 * (s & 1) + j + 1], scale_log2, mc));
        sx += px;
        sy += py;
        pf[s][j] = (bf16)px;
        pf[s][j + 1] = (bf16)py;
      }
    l_run += sx + sy;

    // O^T[d][q] += V^T[d][keys of step s] P^T: 4 dim blocks x 4 key steps
#pragma unroll
    for (int s = 0; s < KTT / 16; ++s) {
      bf16x8 vf[DK / 32];
#pragma unroll
      for (int db = 0; db < DK / 32; ++db) {
        const char *v0 = Vb + s * 16 * 256 + voff[db][0];
        const char *v1 = Vb + s * 16 * 256 + voff[db][1];
        auto lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)v0);
        auto hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)v1);
        __builtin_memcpy(&vf[db], &lo, 8);
        __builtin_memcpy(reinterpret_cast<char *>(&vf[db]) + 8, &hi, 8);
      }
#pragma unroll
      for (int db = 0; db < DK / 32; ++db)
        if (ATTN_ABL & 4)
          oacc[db][s] += (float)vf[db][s & 7] + (float)pf[s][db];
        else
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[db], pf[s], oacc[db], 0, 0, 0);
    }
  };
  // the ring slot of tile kt is kt % NST: the loop walks NST tiles per iteration with constant
  // slots; the last (masked) tile dispatches on its slot
  static_assert(NST == 2 || NST == 3, "ring stages");
  using F = std::false_type;
  using Tr = std::true_type;
  int kt = 0;
#if ATTN_TRACE
  if (NST == 2 && ntiles > 2) {  // the first two tiles apart: prologue latency
    tile(0, std::integral_constant<int, 0>{}, F{});
    tile(1, std::integral_constant<int, 1>{}, F{});
    kt = 2;
  }
  tst[1] = __builtin_readcyclecounter();
#endif
  for (; kt + NST < ntiles; kt += NST) {
    tile(kt, std::integral_constant<int, 0>{}, F{});
    tile(kt + 1, std::integral_constant<int, 1>{}, F{});
    if constexpr (NST == 3) tile(kt + 2, std::integral_constant<int, 2 % NST>{}, F{});
  }
  for (; kt + 1 < ntiles; ++kt) {
    const int sl = kt % NST;
    if (sl == 0)
      tile(kt, std::integral_constant<int, 0>{}, F{});
    else if (NST == 2 || sl == 1)
      tile(kt, std::integral_constant<int, 1>{}, F{});
    else
      tile(kt, std::integral_constant<int, 2 % NST>{}, F{});
  }
  if (ntiles > 0) {
    const int sl = kt % NST;
    if (sl == 0)
      tile(kt, std::integral_constant<int, 0>{}, Tr{});
    else if (NST == 2 || sl == 1)
      tile(kt, std::integral_constant<int, 1>{}, Tr{});
    else
      tile(kt, std::integral_constant<int, 2 % NST>{}, Tr{});
  }

#if ATTN_TRACE
  tst[2] = __builtin_readcyclecounter();
#endif
  // the two halves' sums (same m); O^T[d][query r32], d = 32 db + (r & 3) + 8 (r >> 2) + 4 hh
  {
    auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
    l_run = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  if constexpr (SPL) {
    if (nsp > 1) {
      // the range's partial -> slot (query tile of the sequence, head): piece q4 of every lane
      // contiguous (each store / load of a wave one 1 KiB run; a lane-major image made every
      // instruction 64 partial-line writes)
      const int64_t slot = (int64_t)((cu[b] >> 7) + b + qt) * H + h;  // distinct: see split_layout
      const int S = (T_all + kSplitKeys - 1) / kSplitKeys;             // ranges per slot
      const rsrc_t prs = make_rsrc_any(sa.part, 0x7fffffffu);
      auto pofs = [&](int sr, int q4) {
        return (uint32_t)(((((slot * S + sr) * (kPartLane / 4) + q4) * (64 * NWV) + (64 * w + lane)) * 4) * 4);
      };
#pragma unroll
      for (int db = 0; db < DK / 32; ++db)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                 f32x4{oacc[db][4 * r4], oacc[db][4 * r4 + 1], oacc[db][4 * r4 + 2], oacc[db][4 * r4 + 3]}),
              prs, pofs(s, 4 * db + r4), 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, f32x4{m_run, l_run, 0.f, 0.f}), prs,
          pofs(s, 16), 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __shared__ int last_s;
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(sa.cnt + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int lst = old == nsp - 1;
        if (lst) {
          __hip_atomic_store(sa.cnt + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        last_s = lst;
      }
      __syncthreads();
      if (!last_s) return;
      // merge in range order: M = max_r m_r; O = sum_r O_r 2^((m_r - M) scale); l likewise. The
      // m / l pieces of all ranges, then the O pieces two ranges at a time, loaded ahead of use.
      float M = -INFINITY, mls[kSplitMax][2];
#pragma unroll
      for (int sr = 0; sr < kSplitMax; ++sr) {
        if (sr < nsp) {
          const f32x4 ml = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, pofs(sr, 16), 0, 16));
          mls[sr][0] = ml[0];
          mls[sr][1] = ml[1];
        } else {
          mls[sr][0] = -INFINITY;
          mls[sr][1] = 0.f;
        }
      }
#pragma unroll
      for (int sr = 0; sr < kSplitMax; ++sr) M = max_nn(M, mls[sr][0]);
      float lt = 0.f;
#pragma unroll
      for (int db = 0; db < DK / 32; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] = 0.f;
#pragma unroll
      for (int sr = 0; sr < kSplitMax; sr += 2) {
        if (sr >= nsp) break;
        f32x4 v[2][16];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int q4 = 0; q4 < 16; ++q4)
            v[u][q4] = sr + u < nsp
                           ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, pofs(sr + u, q4), 0, 16))
                           : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float mu = mls[sr + u][0];
          const float a = mu == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((mu - M) * scale_log2);
          lt = __builtin_fmaf(mls[sr + u][1], a, lt);
#pragma unroll
          for (int db = 0; db < DK / 32; ++db)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                oacc[db][4 * r4 + j] = __builtin_fmaf(v[u][4 * db + r4][j], a, oacc[db][4 * r4 + j]);
        }
      }
      l_run = lt;
      m_run = M;
    }
  }
  const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
  if (active && qrow < T && lse != nullptr && hh == 0)
    lse[((int64_t)seq_base + qrow) * H + h] = l_run > 0.f ? m_run * scale_log2 + __log2f(l_run) : INFINITY;
  const rsrc_t orsrc = make_rsrc_any(out, 0x7fffffffu);  // wave-uniform base, per-lane offsets
  if (oflags & 2) {
    // O staged through LDS (the K / V ring is free once every wave has passed this barrier) and
    // stored as whole 256-byte rows, 16 bytes a lane (a lane's own 8-byte pieces of one row per
    // store touched 32 rows per instruction: the store tail was issue-bound). Wave w's 32 x 128
    // tile at w * 8 KiB, 16-byte chunk XOR (row & 15): the column writes 2-way, the row reads
    // conflict-free.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    char *ob = smem + w * (32 * 256);
    if (active) {
#pragma unroll
      for (int db = 0; db < DK / 32; ++db)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          bf16x4 o = {(bf16)(oacc[db][4 * r4] * inv), (bf16)(oacc[db][4 * r4 + 1] * inv),
                      (bf16)(oacc[db][4 * r4 + 2] * inv), (bf16)(oacc[db][4 * r4 + 3] * inv)};
          *reinterpret_cast<bf16x4 *>(ob + r32 * 256 + (((4 * db + r4) ^ (r32 & 15)) << 4) + 8 * hh) = o;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile written (same-wave reads follow)
      const int ch = lane & 15;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = (lane >> 4) + 4 * i, q = q0 + 32 * w + row;
        const uint4 v = *reinterpret_cast<const uint4 *>(ob + row * 256 + ((ch ^ (row & 15)) << 4));
        if (q < T) {
          const uint32_t off = (uint32_t)(((int64_t)seq_base + q) * os + h * DK + ch * 8) * 2u;
          if (oflags & 1)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   orsrc, off, 0, 16);
          else
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   orsrc, off, 0, 0);
        }
      }
    }
  } else if (active && qrow < T) {
    bf16 *orow = out + ((int64_t)seq_base + qrow) * os + h * DK + 4 * hh;
#pragma unroll
    for (int db = 0; db < DK / 32; ++db)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 o = {(bf16)(oacc[db][4 * r4] * inv), (bf16)(oacc[db][4 * r4 + 1] * inv),
                    (bf16)(oacc[db][4 * r4 + 2] * inv), (bf16)(oacc[db][4 * r4 + 3] * inv)};
        if (oflags & 1)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o), orsrc,
                                                (uint32_t)((orow - out) + 32 * db + 8 * r4) * 2u, 0, 16);
        else
          *reinterpret_cast<bf16x4 *>(orow + 32 * db + 8 * r4) = o;
      }
  }
#if ATTN_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tst[3] = __builtin_readcyclecounter();
  if (tid == 0 && blockIdx.x < 4096) {
    unsigned long long *d = g_attn_stamps + blockIdx.x * 8;
    for (int i = 0; i < 4; ++i) d[i] = tst[i];
    d[4] = (unsigned long long)ntiles;
    d[5] = (unsigned long long)(T - q0 < QTW ? T - q0 : QTW);
    d[6] = 1;
  }
#endif
}

// The key-split work list of a packed layout: for every sequence b (len = cu[b+1] - cu[b] > 0),
// heads h, query tiles qt < ceil(len / 128) and ranges s < ceil(len / kSplitKeys) (1 when len <=
// kSplitKeys): one item, in (b, h, qt, s) order; *count = their number. ONE wave: a shuffle scan
// over 64 sequences at a time (a 1024-thread block scan with its barriers took ~10 us in the graph).
__global__ __launch_bounds__(64) void attn_items_kernel(const int32_t *__restrict__ cu, int B, int H,
                                                        int *__restrict__ items, int *__restrict__ count, int cap,
                                                        int *__restrict__ cnt, int slots) {
  const int lane = threadIdx.x;
  for (int i = lane; i < slots; i += 64) cnt[i] = 0;  // the arrival counters start at zero
  int carry = 0;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + lane;
    int nq = 0, ns = 1;
    if (b < B) {
      const int len = cu[b + 1] - cu[b];
      nq = len > 0 ? (len + 127) / 128 : 0;
      ns = len > kSplitKeys ? (len + kSplitKeys - 1) / kSplitKeys : 1;
    }
    const int n = nq * ns * H;
    int inc = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    const int off = carry + inc - n;
    for (int h = 0; h < H; ++h)
      for (int qt = 0; qt < nq; ++qt)
        for (int s = 0; s < ns; ++s) {
          const int i = off + (h * nq + qt) * ns + s;
          if (i < cap) items[i] = (b << 16) | (qt << 8) | (s << 4) | h;
        }
    carry += __shfl(inc, 63, 64);
  }
  if (lane == 0) *count = carry < cap ? carry : cap;
}

}  // namespace

// the key-split workspace: [count, pad][items: cap][arrival counters: slots][partials: slots x S
// ranges]. A slot is (cu[b] >> 7) + b + qt per sequence query tile and head: distinct, and below
// (rows_max / 128 + B + ceil(T / 128)) * H when cu[B] <= rows_max; items <= that many x S.
struct SplitLayout {
  int64_t slots, cap, items_off, cnt_off, part_off, bytes;
};
static SplitLayout split_layout(int B, int T, int H, int64_t rows_max) {
  SplitLayout l;
  const int S = (T + kSplitKeys - 1) / kSplitKeys;
  l.slots = (rows_max / 128 + B + (T + 127) / 128) * (int64_t)H;
  l.cap = l.slots * S;
  l.items_off = 256;
  l.cnt_off = (l.items_off + l.cap * 4 + 255) / 256 * 256;
  l.part_off = (l.cnt_off + l.slots * 4 + 255) / 256 * 256;
  l.bytes = l.part_off + l.slots * S * 256 * kPartLane * 4;
  return l;
}

static int attention_launch(const void *qkv, int dtype, int64_t qkv_row_stride, const int64_t *key_lens, int B, int T,
                            int H, int dk, float temperature, void *out, int64_t out_row_stride,
                            const int32_t *seq_cu, float *lse, int waves, void *split_ws, int64_t split_ws_bytes,
                            int64_t rows_max, fs2_stream_t stream) {
  if (qkv == nullptr || (key_lens == nullptr && seq_cu == nullptr) || out == nullptr) return FS2_EINVAL;
  if (dk != DK || H <= 0 || B < 0 || T < 0 || !(temperature > 0.f)) return FS2_EINVAL;
  if (qkv_row_stride < 3LL * H * dk || out_row_stride < (int64_t)H * dk) return FS2_EINVAL;
  const int ce = dtype == FS2_BF16 ? 8 : 4;
  if ((qkv_row_stride % ce) != 0) return FS2_EINVAL;
  if (B == 0 || T == 0) return FS2_OK;
  const float scale_log2 = 1.4426950408889634f / temperature;
  dim3 grid((T + QT - 1) / QT, H, B);
  hipStream_t s = as_stream(stream);
  if (dtype == FS2_BF16) {
    const int64_t bytes = (int64_t)B * T * qkv_row_stride * 2;
    if (bytes >= (1LL << 31) || (out_row_stride & 3)) return FS2_EUNSUPPORTED;
    // 8 waves (128 queries) share each K/V tile for sequences longer than 64; 4 waves otherwise
    // (encoder, L <= 64: a 128-query workgroup would idle half its waves). 2-stage K/V ring: at the
    // cfg2 decoder shape (packed, ~390 frames) 16 waves per CU (2 workgroups) hide the MFMA ->
    // softmax -> MFMA chain better than a deeper ring at 8 waves per CU (29.9 us vs 35.0 us with 3
    // stages; 4 waves / 2 or 3 stages 34.5 / 49.9 us; the software-pipelined, 32-key-tile and
    // 32-queries-per-wave variants measured 30.5, 31-32 and 27.4 us standalone / bench-neutral and
    // were removed in round 3).
    static const int use32 = [] {
      const char *e = getenv("FS2_ATTN32");
      return (e != nullptr && e[0] == '0') ? 0 : 1;
    }();
    // output stores: bit 0 write-through (sc1: the lines leave L2; FS2_OUT_SC1=0 plain, A/B), bit 1
    // rows staged through LDS (FS2_ATTN_OSTAGE=0 stores a lane's 8-byte pieces directly, A/B)
    static const int oflags = [] {
      const char *e = getenv("FS2_OUT_SC1"), *f = getenv("FS2_ATTN_OSTAGE");
      return ((e != nullptr && e[0] == '0') ? 0 : 1) | ((f != nullptr && f[0] == '0') ? 0 : 2);
    }();
    // waves x K/V ring stages: 4x2, or 8x2 when the caller says the sequences are long and dense
    // (fs2_attention_ex waves = 8: the cfg2 decoder, ~390 of T = 430 frames each: 145.2 vs
    // 148.4-149.3 us of decoder attention per forward, same box). With a long max length over short
    // sequences (free-running cfg2: T 960, mean 174 frames) the 256-query tiles leave most
    // (utterance, head) pairs ONE workgroup (forced 8x2: 1.2845 vs 1.2253 ms per call), and cfg4
    // (8.58 vs 8.49 ms); the kernel sees only T, so the caller decides. FS2_ATTN32_FORM=4x2 / 8x2 /
    // 8x3 overrides (8x3: 25.4-26.2 us at cfg2).
    static const int form_env = [] {
      const char *e = getenv("FS2_ATTN32_FORM");
      return e == nullptr ? -1 : (e[0] == '8' && e[2] == '3') ? 2 : (e[0] == '8') ? 1 : 0;
    }();
    const int form32 = form_env >= 0 ? form_env : (waves == 8 ? 1 : 0);
    if (split_ws != nullptr && use32) {
      // the key-split form over the layout's work list (fs2_attention_items)
      if (seq_cu == nullptr || lse != nullptr || T <= kSplitKeys || (T + kSplitKeys - 1) / kSplitKeys > kSplitMax ||
          H > 16 || rows_max <= 0 || rows_max > (int64_t)B * T)
        return FS2_EINVAL;
      const SplitLayout l = split_layout(B, T, H, rows_max);
      if (split_ws_bytes < l.bytes) return FS2_EINVAL;
      if (l.bytes - l.part_off >= (1LL << 31) || l.cap >= (1LL << 31) - 64) return FS2_EUNSUPPORTED;
      char *w0 = static_cast<char *>(split_ws);
      SplitArgs sa{reinterpret_cast<const int *>(w0 + l.items_off), reinterpret_cast<const int *>(w0),
                   reinterpret_cast<float *>(w0 + l.part_off), reinterpret_cast<int *>(w0 + l.cnt_off)};
      const int64_t nwg = (l.cap + 31) / 32 * 32;  // whole groups of 4 items per XCD
      hipLaunchKernelGGL((attn32_kernel<4, 2, true>), dim3((unsigned)nwg), dim3(256), 0, s,
                         reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H,
                         (T + 127) / 128, scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse,
                         oflags, sa);
    } else if (T > 64 && use32 && form32 == 0) {
      // 4 waves x 32 queries, two workgroups per CU (2 x 64 KiB of K / V ring)
      const int nqt = (T + 127) / 128;
      hipLaunchKernelGGL((attn32_kernel<4, 2>), dim3(nqt * H * B), dim3(256), 0, s,
                         reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H, nqt,
                         scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse, oflags);
    } else if (T > 64 && use32) {
      // 8 waves x 32 queries: each K / V tile serves 256 queries (half the K / V traffic per query)
      const int nqt = (T + 255) / 256;
      if (form32 == 1)
        hipLaunchKernelGGL((attn32_kernel<8, 2>), dim3(nqt * H * B), dim3(512), 0, s,
                           reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H, nqt,
                           scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse, oflags);
      else
        hipLaunchKernelGGL((attn32_kernel<8, 3>), dim3(nqt * H * B), dim3(512), 0, s,
                           reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H, nqt,
                           scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse, oflags);
    } else if (T > 64) {
      const int nqt = (T + 127) / 128;
      hipLaunchKernelGGL((attn_bf16_kernel<8, 2>), dim3(nqt * H * B), dim3(512), 0, s,
                         reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H, nqt,
                         scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse);
    } else {
      const int nqt = (T + 63) / 64;
      hipLaunchKernelGGL((attn_bf16_kernel<4, 2>), dim3(nqt * H * B), dim3(256), 0, s,
                         reinterpret_cast<const bf16 *>(qkv), qkv_row_stride, (uint32_t)bytes, key_lens, B, T, H, nqt,
                         scale_log2, reinterpret_cast<bf16 *>(out), out_row_stride, seq_cu, lse);
    }
  } else if (dtype == FS2_F32)
    hipLaunchKernelGGL(attn_kernel<FS2_F32>, grid, dim3(256), 0, s, reinterpret_cast<const float *>(qkv),
                       qkv_row_stride, key_lens, T, H, scale_log2, reinterpret_cast<float *>(out), out_row_stride,
                       seq_cu, lse);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_attention(const void *qkv, int dtype, int64_t qkv_row_stride, const int64_t *key_lens, int B, int T,
                             int H, int dk, float temperature, void *out, int64_t out_row_stride,
                             const int32_t *seq_cu, float *lse, fs2_stream_t stream) {
  return attention_launch(qkv, dtype, qkv_row_stride, key_lens, B, T, H, dk, temperature, out, out_row_stride, seq_cu,
                          lse, 0, nullptr, 0, 0, stream);
}

extern "C" int fs2_attention_ex(const void *qkv, int dtype, int64_t qkv_row_stride, const int64_t *key_lens, int B,
                                int T, int H, int dk, float temperature, void *out, int64_t out_row_stride,
                                const int32_t *seq_cu, float *lse, int waves, void *split_ws, int64_t split_ws_bytes,
                                int64_t rows_max, fs2_stream_t stream) {
  if (waves != 0 && waves != 4 && waves != 8) return FS2_EINVAL;
  return attention_launch(qkv, dtype, qkv_row_stride, key_lens, B, T, H, dk, temperature, out, out_row_stride, seq_cu,
                          lse, waves, split_ws, split_ws_bytes, rows_max, stream);
}

extern "C" int64_t fs2_attention_split_ws_bytes(int B, int T, int H, int64_t rows_max) {
  if (B <= 0 || T <= kSplitKeys || (T + kSplitKeys - 1) / kSplitKeys > kSplitMax || H <= 0 || H > 16 || rows_max <= 0)
    return 0;
  return split_layout(B, T, H, rows_max).bytes;
}

extern "C" int fs2_attention_items(const int32_t *seq_cu, int B, int T, int H, void *split_ws, int64_t split_ws_bytes,
                                   int64_t rows_max, fs2_stream_t stream) {
  if (seq_cu == nullptr || split_ws == nullptr || B <= 0 || B >= 32768 || T <= kSplitKeys || T > 256 * 128 ||
      H <= 0 || H > 16 || rows_max <= 0 || rows_max > (int64_t)B * T)
    return FS2_EINVAL;
  const SplitLayout l = split_layout(B, T, H, rows_max);
  if (split_ws_bytes < l.bytes) return FS2_EINVAL;
  char *w0 = static_cast<char *>(split_ws);
  hipLaunchKernelGGL(attn_items_kernel, dim3(1), dim3(64), 0, as_stream(stream), seq_cu, B, H,
                     reinterpret_cast<int *>(w0 + l.items_off), reinterpret_cast<int *>(w0), (int)l.cap,
                     reinterpret_cast<int *>(w0 + l.cnt_off), (int)l.slots);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
