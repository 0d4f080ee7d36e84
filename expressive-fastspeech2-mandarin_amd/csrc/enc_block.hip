// The encoder's attention sub-layer as ONE launch per layer (gfx950 / CDNA4):
//
//   qkv = x Wqkv^T + bqkv                                  (transformer/SubLayers.py:39-41)
//   o   = softmax(q k^T / temperature, keys < len) v       (transformer/Modules.py:14-25, 2 heads)
//   h   = masked_fill(LayerNorm(o Wfc^T + bfc + x), t >= len, 0)   (SubLayers.py:54-55, Layers.py:25)
//
// The encoder's rows are short ([B, L <= 64] phonemes): as three launches (the weight-resident
// Q|K|V GEMM, attention, the fc + LN GEMM) each one pays a launch, a prologue and an HBM round trip
// of its 4k-row operands for ~1-8 GFLOP -- 22.5 us per layer at cfg2 for ~38 MFLOP per utterance.
// Here one workgroup owns one utterance: its x tile is DMA'd to LDS once, Q | K | V never leave
// LDS, the attention output stays there for the fc GEMM, and only h is written.
//
// 8 waves (two per SIMD). Phase 1 (Q|K|V): wave w computes output columns 96w .. 96w+95 (6 blocks
// of 16) x 64 rows with the weights streamed from the fragment-ordered buffer (ops.pack_frag_rows,
// 16-byte loads straight into A-operand registers, a 4-k-step register ring) and x fragments from
// LDS; the epilogue (+ bias, bf16) writes Q row-major and K / V in attention.hip's swizzled image.
// Phase 2: wave w = (head w / 4, 16 queries) runs attn_bf16_kernel's per-wave arithmetic on the
// single 64-key tile (S^T = K Q^T, lane-local softmax, O^T = V^T P^T with transposed V reads), so
// q / k / v / o round exactly as the three-launch path does. Phase 3: wave w computes fc columns
// 32w .. 32w+31, then + bfc + x, LayerNorm statistics over the 8 waves through LDS, the row mask,
// and whole-row stores through an LDS staging tile.
#include "cond.h"
#include "fs2_common.h"

namespace {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int D = 256, NQKV = 768, LMAX = 64, DK = 128, NT = 512;
constexpr int kUnit = 4096;  // fragment-order unit: 64 weight rows x 32 channels

__device__ __forceinline__ rsrc_t rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
// attention.hip's K / V image: 256-byte rows (one head's 128 dims), 16-byte chunks XOR-swizzled
__device__ __forceinline__ int kv_swz(int row) { return ((row & 7) << 1) | ((row >> 3) & 1); }
__device__ __forceinline__ int kv_off(int row, int chunk) { return row * 256 + ((chunk ^ kv_swz(row)) << 4); }
__device__ __forceinline__ float max_nn(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float rows_sum(float v) {  // over the 4 lane groups of one column
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

// workgroup barrier WITHOUT the vmcnt drain __syncthreads() implies (the weight loads in flight
// across it), after this wave's LDS traffic retired
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct EncBlockArgs {
  const bf16 *x;       // [B, L, 256]
  const int64_t *lens; // [B]
  int B, L;
  const bf16 *wqkv;    // pack_frag_rows([768, 256])
  const float *bqkv;   // [768]
  const bf16 *wfc;     // pack_frag_rows([256, 256])
  const float *bfc, *gamma, *beta;
  float eps, scale_log2;
  bf16 *out;           // [B, L, 256]
  // EMBED (the first encoder block): x = bf16(emb[tokens] + pe) built in LDS (fs2_embed_pe's
  // arithmetic: out-of-vocabulary ids give NaN rows and count in *bad), and the forward's masks
  // get_mask_from_lengths(lens, L) / (mel_lens, T_mel) written beside it (NULL: not wanted)
  const int64_t *tokens;
  const float *emb, *pe;
  int vocab, T_mel;
  int32_t *bad;
  uint8_t *src_mask;
  const int64_t *mel_lens;
  uint8_t *mel_mask;
  // head-split form (enc_attn_half_kernel): per-utterance arrival counters (zero between
  // launches; the last arriver resets) and the f32 partial fc rows, 64 KiB per (utterance, head)
  int *cnt;
  char *part;
  uint32_t part_bytes;
  // EMBED: workgroups B .. B + ncond - 1 compute the conditioning vectors (cond.h tiles, ncx per row)
  CondArgs cond;
  int ncond, ncx;
};

// LDS image (bytes)
constexpr int XP = D * 2 + 16;                  // x / o / staging row pitch: 16 rows' B-fragment reads hit distinct banks
constexpr int QP = DK * 2 + 16;                 // Q rows (per head)
constexpr int X_OFF = 0;                        // x tile [64][XP]; later the output staging tile
constexpr int Q_OFF = X_OFF + LMAX * XP;        // Q [2][64][QP]; later o [64][XP]
constexpr int K_OFF = Q_OFF + 2 * LMAX * QP;    // K [2][64 x 256 B] (kv_off)
constexpr int V_OFF = K_OFF + 2 * LMAX * 256;   // V [2][64 x 256 B]
constexpr int RED_OFF = V_OFF + 2 * LMAX * 256; // LayerNorm partials [2 passes][64 rows][8 waves] f32
constexpr int VEC_OFF = RED_OFF + 2 * LMAX * 8 * 4; // bqkv (768) | bfc | gamma | beta (256 each) f32
constexpr int SMEM = VEC_OFF + (NQKV + 3 * D) * 4;
static_assert(2 * LMAX * QP >= LMAX * XP, "o fits the Q region");
static_assert(SMEM <= 163840, "LDS");

#ifndef ENC_TRACE
#define ENC_TRACE 0  // analysis builds only: wave 0's shader clock at each phase into the workspace tail
#endif

// the conditioning tiles out of line: inlined, their registers inflated the block's allocation
__device__ __attribute__((noinline)) void cond_role(const CondArgs &a, int bx, int by, int tid, float *sm) {
  cond_tile(a, bx, by, tid, sm);
}

template <bool EMBED, bool COND = false>
__global__ __launch_bounds__(NT, 1) void enc_attn_block_kernel(EncBlockArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  uint64_t tst[10];
  int ntst = 0;
  auto stamp = [&]() {
    if (ENC_TRACE) {
      __builtin_amdgcn_sched_barrier(0);
      tst[ntst++] = __builtin_readcyclecounter();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp();
  const int tid = threadIdx.x, lane = tid & 63;
  if constexpr (COND) {
    if ((int)blockIdx.x >= p.B) {  // a conditioning-vector tile on an otherwise idle CU
      const int c = (int)blockIdx.x - p.B;
      cond_role(p.cond, c % p.ncx, c / p.ncx, tid, reinterpret_cast<float *>(smem));
      return;
    }
  }
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.x, L = p.L;
  const int64_t len64 = p.lens[b];
  const int len = (int)(len64 < 0 ? 0 : (len64 > L ? L : len64));
  const uint32_t xrow0 = (uint32_t)b * (uint32_t)L;

  // ---- x tile (rows >= L: zeros) and the four vectors by LDS-DMA; Q|K|V weight ring start
  static_assert(LMAX * XP % 1024 == 0, "whole 1 KiB pieces");
  if constexpr (!EMBED) {
    const rsrc_t xr = rsrc(p.x, (uint32_t)p.B * (uint32_t)L * D * 2u);
    for (int pc = w; pc < LMAX * XP / 1024; pc += 8) {
      const int o = pc * 1024 + lane * 16, r = o / XP, within = o - r * XP;
      const bool ok = r < L && within < D * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                               16, ok ? (xrow0 + r) * (uint32_t)(D * 2) + (uint32_t)within : 0x80000000u,
                                               0, 0, 0);
    }
  }
  {  // 6 KiB of vectors = 6 pieces: bqkv (3), bfc, gamma, beta
    if (w < 6) {
      const float *src = w < 3 ? p.bqkv + 256 * w : w == 3 ? p.bfc : w == 4 ? p.gamma : p.beta;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(src, 1024), (__attribute__((address_space(3))) void *)(smem + VEC_OFF + w * 1024),
                                               16, (uint32_t)lane * 16u, 0, 0, 0);
    }
  }
  const float *vqkv = reinterpret_cast<const float *>(smem + VEC_OFF);
  const float *vfc = vqkv + NQKV, *vg = vfc + D, *vb = vg + D;

  // ---- phase 1: Q|K|V. Output block nb (16 columns) = rows 16 (nb & 3) of weight quad nb >> 2
  constexpr int NB1 = 6, RING = 4;
  const rsrc_t wq = rsrc(p.wqkv, (uint32_t)NQKV * D * 2u);
  bf16x8 ring[RING][NB1];
  auto wload = [&](int ks, bf16x8 (&dst)[NB1]) {
    // pinned after the MFMAs that read the slot (hipcc otherwise sinks the refills below every
    // MFMA of the first four k-steps, and k-steps 4..7 then wait out a full L2 round trip)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NB1; ++i) {
      const int nb = NB1 * w + i;
      auto v = __builtin_amdgcn_raw_buffer_load_b128(
          wq, (uint32_t)lane * 16u + (uint32_t)(nb & 3) * 1024u, (uint32_t)(((nb >> 2) * (D / 32) + ks) * kUnit), 0);
      dst[i] = __builtin_bit_cast(bf16x8, v);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int ks = 0; ks < RING; ++ks) wload(ks, ring[ks]);
  if constexpr (EMBED) {
    // x rows (transformer/Models.py:82-91): row r, 8-channel chunk c per item, 4 items a thread
    for (int i = tid; i < LMAX * (D / 8); i += NT) {
      const int r = i >> 5, c = (i & 31) * 8;
      bf16x8 o;
      if (r < L) {
        const int64_t tok = p.tokens[xrow0 + r];
        if (tok < 0 || tok >= p.vocab) {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)__builtin_nanf("");
          if (p.bad != nullptr && c == 0) atomicAdd(p.bad, 1);
        } else {
          float v[8], e[8];
          load8(p.emb + tok * D + c, v);
          load8(p.pe + (int64_t)r * D + c, e);
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)(v[q] + e[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = (bf16)0.f;
      }
      *reinterpret_cast<bf16x8 *>(smem + X_OFF + r * XP + c * 2) = o;
    }
    // get_mask_from_lengths (utils/tools.py:152-160): True = padding
    if (p.src_mask != nullptr)
      for (int t = tid; t < L; t += NT) p.src_mask[(int64_t)b * L + t] = (int64_t)t >= len64 ? 1 : 0;
    if (p.mel_mask != nullptr) {
      const int64_t ml = p.mel_lens[b];
      for (int t = tid; t < p.T_mel; t += NT) p.mel_mask[(int64_t)b * p.T_mel + t] = (int64_t)t >= ml ? 1 : 0;
    }
  }
  // x tile, vectors and k-step 0 landed (k-steps 1..3, the youngest 3 x NB1 loads, may stay in
  // flight: waiting for the whole ring made every CU pull ~230 KB before its first MFMA)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((RING - 1) * NB1) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();
  stamp();

  f32x4 acc[NB1][4];
#pragma unroll
  for (int i = 0; i < NB1; ++i)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[i][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    bf16x8 xf[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      xf[mb] = *reinterpret_cast<const bf16x8 *>(smem + X_OFF + (16 * mb + li) * XP + ks * 64 + g * 16);
#pragma unroll
    for (int i = 0; i < NB1; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        acc[i][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[ks % RING][i], xf[mb], acc[i][mb], 0, 0, 0);
    if (ks + RING < D / 32) wload(ks + RING, ring[ks % RING]);
  }
  stamp();
  // + bias, bf16: lane holds columns n = 16 nb + 4 g + j of row m = 16 mb + li
#pragma unroll
  for (int i = 0; i < NB1; ++i) {
    const int n = 16 * (NB1 * w + i) + 4 * g;
    const float4 bb = *reinterpret_cast<const float4 *>(vqkv + n);
    const int part = n >> 8, hh = (n >> 7) & 1, dim = n & 127;  // part 0 Q, 1 K, 2 V
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m = 16 * mb + li;
      const f32x4 v = acc[i][mb];
      const bf16x4 o = {(bf16)(v[0] + bb.x), (bf16)(v[1] + bb.y), (bf16)(v[2] + bb.z), (bf16)(v[3] + bb.w)};
      char *dst = part == 0 ? smem + Q_OFF + (hh * LMAX + m) * QP + dim * 2
                            : smem + (part == 1 ? K_OFF : V_OFF) + hh * LMAX * 256 + kv_off(m, dim >> 3) + (dim & 7) * 2;
      *reinterpret_cast<bf16x4 *>(dst) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();

  // fc weights for this wave's two column blocks, all 8 k-steps (64 VGPRs): in flight during attention
  const rsrc_t wf = rsrc(p.wfc, (uint32_t)D * D * 2u);
  bf16x8 fw[D / 32][2];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int nb = 2 * w + i;
      fw[ks][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                 wf, (uint32_t)lane * 16u + (uint32_t)(nb & 3) * 1024u,
                                                 (uint32_t)(((nb >> 2) * (D / 32) + ks) * kUnit), 0));
    }
  stamp();
  // ---- phase 2: attention, wave w = head w >> 2, queries 16 (w & 3) + li (attn_bf16_kernel's
  // per-wave arithmetic on one 64-key tile: keys >= len at -inf)
  const int h = w >> 2, qb = w & 3;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = *reinterpret_cast<const bf16x8 *>(smem + Q_OFF + (h * LMAX + 16 * qb + li) * QP + (32 * s + 8 * g) * 2);
  f32x4 oacc[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float l_run = 0.f;
  if (len > 0) {
    const char *Kb = smem + K_OFF + h * LMAX * 256;
    const char *Vb = smem + V_OFF + h * LMAX * 256;
    constexpr int NBK = LMAX / 16;
    f32x4 sacc[NBK];
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni) {
      sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(Kb + kv_off(ni * 16 + li, 4 * s + g));
        sacc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sacc[ni], 0, 0, 0);
      }
    }
    const int lim = len - 4 * g;  // scores of query li: keys ni*16 + 4g + j
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ni * 16 + j >= lim) sacc[ni][j] = -INFINITY;
    float mx = -INFINITY;
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni) {
      mx = max_nn(max_nn(mx, sacc[ni][0]), sacc[ni][1]);
      mx = max_nn(max_nn(mx, sacc[ni][2]), sacc[ni][3]);
    }
    const float m_new = rows_max(mx);
    const float mc = -m_new * p.scale_log2;
    float sx = 0.f, sy = 0.f;
    bf16x8 pf[NBK / 2];
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const float px = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp], p.scale_log2, mc));
        const float py = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp + 1], p.scale_log2, mc));
        sx += px;
        sy += py;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp] = (bf16)px;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp + 1] = (bf16)py;
      }
    l_run = rows_sum(sx + sy);
    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int s2 = 0; s2 < NBK / 2; ++s2) {
#pragma unroll
      for (int h4 = 0; h4 < DK / 64; ++h4) {
        bf16x8 vf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int nd = 4 * h4 + i;
          const char *vp = Vb + kv_off(4 * g + tq, nd * 2 + (tp >> 1)) + (tp & 1) * 8 + s2 * 32 * 256;
          auto lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)vp);
          auto hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(vp + 16 * 256));
          __builtin_memcpy(&vf[i], &lo, 8);
          __builtin_memcpy(reinterpret_cast<char *>(&vf[i]) + 8, &hi, 8);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          oacc[4 * h4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[i], pf[s2], oacc[4 * h4 + i], 0, 0, 0);
      }
    }
  }
  stamp();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();  // every wave holds its Q fragments: the Q region becomes o
  {
    // O^T[d = nd*16 + 4g + j][query li] -> o[query][h*128 + d] (bf16, as the attention launch writes)
    const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
    const int q = 16 * qb + li;
#pragma unroll
    for (int nd = 0; nd < DK / 16; ++nd) {
      const bf16x4 o = {(bf16)(oacc[nd][0] * inv), (bf16)(oacc[nd][1] * inv), (bf16)(oacc[nd][2] * inv),
                        (bf16)(oacc[nd][3] * inv)};
      *reinterpret_cast<bf16x4 *>(smem + Q_OFF + q * XP + (h * DK + nd * 16 + 4 * g) * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();  // o complete

  stamp();
  // ---- phase 3: fc + bfc + x, LayerNorm, row mask
  f32x4 fa[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) fa[i][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    bf16x8 of[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      of[mb] = *reinterpret_cast<const bf16x8 *>(smem + Q_OFF + (16 * mb + li) * XP + ks * 64 + g * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) fa[i][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks][i], of[mb], fa[i][mb], 0, 0, 0);
  }
  stamp();
  // v = fc + bfc + x; per-row partial sums over this wave's 32 columns
  float* red = reinterpret_cast<float *>(smem + RED_OFF);
  float part[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = 16 * mb + li;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = 16 * (2 * w + i) + 4 * g;
      const float4 bb = *reinterpret_cast<const float4 *>(vfc + n);
      const bf16x4 xv = *reinterpret_cast<const bf16x4 *>(smem + X_OFF + m * XP + n * 2);
      f32x4 v = fa[i][mb];
      v[0] = v[0] + bb.x + (float)xv[0];
      v[1] = v[1] + bb.y + (float)xv[1];
      v[2] = v[2] + bb.z + (float)xv[2];
      v[3] = v[3] + bb.w + (float)xv[3];
      fa[i][mb] = v;
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    part[mb] = rows_sum(s);
  }
  // across the 8 waves through LDS; the two passes use separate slots (one barrier each)
  auto reduce = [&](float (&pv)[4], float (&tot)[4], int pass) {
    float *rb = red + pass * LMAX * 8;
    if (g == 0) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) rb[(16 * mb + li) * 8 + w] = pv[mb];
    }
    bar();
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const float4 a = *reinterpret_cast<const float4 *>(rb + (16 * mb + li) * 8);
      const float4 c = *reinterpret_cast<const float4 *>(rb + (16 * mb + li) * 8 + 4);
      tot[mb] = ((a.x + a.y) + (a.z + a.w)) + ((c.x + c.y) + (c.z + c.w));
    }
  };
  float mean[4], var[4];
  reduce(part, mean, 0);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    mean[mb] *= 1.0f / D;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 d = fa[i][mb];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] -= mean[mb];
      fa[i][mb] = d;
      s += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
    }
    part[mb] = rows_sum(s);
  }
  reduce(part, var, 1);  // (its barrier also retires every wave's x reads: X becomes the staging tile)
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = 16 * mb + li;
    const float rstd = 1.0f / sqrtf(var[mb] * (1.0f / D) + p.eps);
    const float keep = m < len ? 1.0f : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = 16 * (2 * w + i) + 4 * g;
      const float4 gg = *reinterpret_cast<const float4 *>(vg + n);
      const float4 be = *reinterpret_cast<const float4 *>(vb + n);
      const f32x4 d = fa[i][mb];
      const bf16x4 o = {(bf16)((d[0] * rstd * gg.x + be.x) * keep), (bf16)((d[1] * rstd * gg.y + be.y) * keep),
                        (bf16)((d[2] * rstd * gg.z + be.z) * keep), (bf16)((d[3] * rstd * gg.w + be.w) * keep)};
      *reinterpret_cast<bf16x4 *>(smem + X_OFF + m * XP + n * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();
  stamp();
  // whole rows (32 x 16 B each) of the L valid positions
  uint4 *orow = reinterpret_cast<uint4 *>(p.out + (size_t)xrow0 * D);
  for (int i = tid; i < L * (D * 2 / 16); i += NT) {
    const int m = i >> 5, c = i & 31;
    orow[i] = *reinterpret_cast<const uint4 *>(smem + X_OFF + m * XP + c * 16);
  }
  stamp();
  if (ENC_TRACE && tid == 0 && p.cnt != nullptr) {
    uint64_t *o = reinterpret_cast<uint64_t *>(p.part + p.part_bytes - 65536u) + 16 * blockIdx.x;
    for (int i = 0; i < ntst; ++i) o[i] = tst[i];
    o[15] = (uint64_t)ntst;
  }
}


// ---------------------------------------------------------------------------------------------
// Head-split form: TWO workgroups per utterance, one per head, so the 512 KB of weights an
// utterance needs stream into two CUs (256 KB each) and the 128 launched workgroups spread the
// L2 traffic that bounds the one-workgroup form (16.4 us per layer on 64 CUs). Workgroup (b, h):
// Q_h | K_h | V_h (384 columns: 8 waves x 3 blocks), head h's attention (waves 0-3, as above),
// and its half of the fc GEMM, fc_h = o_h Wfc[:, 128h .. 128h+127]^T (K = 128): the two halves
// meet through a sc1 hand-off in the split-K workspace (as fs2_ffn's split form: write-through
// stores, drain, one counter add; the last arriver sums head 0 + head 1 in that order, adds bfc
// and x and runs the LayerNorm). A pair shares an XCD (bid = 16 G + 8 h + x: utterance 8 G + x).
template <bool EMBED>
__global__ __launch_bounds__(NT, 1) void enc_attn_half_kernel(EncBlockArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int bid = blockIdx.x, hh = (bid >> 3) & 1, b = (bid >> 4) * 8 + (bid & 7), L = p.L;
  if (b >= p.B) return;
  const int64_t len64 = p.lens[b];
  const int len = (int)(len64 < 0 ? 0 : (len64 > L ? L : len64));
  const uint32_t xrow0 = (uint32_t)b * (uint32_t)L;

  if constexpr (!EMBED) {
    const rsrc_t xr = rsrc(p.x, (uint32_t)p.B * (uint32_t)L * D * 2u);
    for (int pc = w; pc < LMAX * XP / 1024; pc += 8) {
      const int o = pc * 1024 + lane * 16, r = o / XP, within = o - r * XP;
      const bool ok = r < L && within < D * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                               16, ok ? (xrow0 + r) * (uint32_t)(D * 2) + (uint32_t)within : 0x80000000u,
                                               0, 0, 0);
    }
  }
  if (w < 6) {
    const float *src = w < 3 ? p.bqkv + 256 * w : w == 3 ? p.bfc : w == 4 ? p.gamma : p.beta;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(src, 1024), (__attribute__((address_space(3))) void *)(smem + VEC_OFF + w * 1024),
                                             16, (uint32_t)lane * 16u, 0, 0, 0);
  }
  const float *vqkv = reinterpret_cast<const float *>(smem + VEC_OFF);
  const float *vfc = vqkv + NQKV, *vg = vfc + D, *vb = vg + D;

  // ---- Q_h | K_h | V_h: local block j = 3w + i (0..23) -> part j / 8, global block 16 part + 8 hh + j % 8
  constexpr int NB1 = 3, RING = 4;
  const rsrc_t wq = rsrc(p.wqkv, (uint32_t)NQKV * D * 2u);
  bf16x8 ring[RING][NB1];
  auto gblock = [&](int i) {
    const int j = NB1 * w + i;
    return 16 * (j >> 3) + 8 * hh + (j & 7);
  };
  auto wload = [&](int ks, bf16x8 (&dst)[NB1]) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NB1; ++i) {
      const int nb = gblock(i);
      auto v = __builtin_amdgcn_raw_buffer_load_b128(
          wq, (uint32_t)lane * 16u + (uint32_t)(nb & 3) * 1024u, (uint32_t)(((nb >> 2) * (D / 32) + ks) * kUnit), 0);
      dst[i] = __builtin_bit_cast(bf16x8, v);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int ks = 0; ks < RING; ++ks) wload(ks, ring[ks]);
  if constexpr (EMBED) {
    for (int i = tid; i < LMAX * (D / 8); i += NT) {
      const int r = i >> 5, c = (i & 31) * 8;
      bf16x8 o;
      if (r < L) {
        const int64_t tok = p.tokens[xrow0 + r];
        if (tok < 0 || tok >= p.vocab) {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)__builtin_nanf("");
          if (p.bad != nullptr && c == 0 && hh == 0) atomicAdd(p.bad, 1);
        } else {
          float v[8], e[8];
          load8(p.emb + tok * D + c, v);
          load8(p.pe + (int64_t)r * D + c, e);
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)(v[q] + e[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = (bf16)0.f;
      }
      *reinterpret_cast<bf16x8 *>(smem + X_OFF + r * XP + c * 2) = o;
    }
    if (hh == 0) {
      if (p.src_mask != nullptr)
        for (int t = tid; t < L; t += NT) p.src_mask[(int64_t)b * L + t] = (int64_t)t >= len64 ? 1 : 0;
      if (p.mel_mask != nullptr) {
        const int64_t ml = p.mel_lens[b];
        for (int t = tid; t < p.T_mel; t += NT) p.mel_mask[(int64_t)b * p.T_mel + t] = (int64_t)t >= ml ? 1 : 0;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((RING - 1) * NB1) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();

  f32x4 acc[NB1][4];
#pragma unroll
  for (int i = 0; i < NB1; ++i)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[i][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    bf16x8 xf[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      xf[mb] = *reinterpret_cast<const bf16x8 *>(smem + X_OFF + (16 * mb + li) * XP + ks * 64 + g * 16);
#pragma unroll
    for (int i = 0; i < NB1; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        acc[i][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[ks % RING][i], xf[mb], acc[i][mb], 0, 0, 0);
    if (ks + RING < D / 32) wload(ks + RING, ring[ks % RING]);
  }
  // + bias, bf16 -> Q (head slot 0 of the Q region) / K / V images of this head
#pragma unroll
  for (int i = 0; i < NB1; ++i) {
    const int n = 16 * gblock(i) + 4 * g;
    const float4 bb = *reinterpret_cast<const float4 *>(vqkv + n);
    const int part = n >> 8, dim = n & 127;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m = 16 * mb + li;
      const f32x4 v = acc[i][mb];
      const bf16x4 o = {(bf16)(v[0] + bb.x), (bf16)(v[1] + bb.y), (bf16)(v[2] + bb.z), (bf16)(v[3] + bb.w)};
      char *dst = part == 0 ? smem + Q_OFF + m * QP + dim * 2
                            : smem + (part == 1 ? K_OFF : V_OFF) + kv_off(m, dim >> 3) + (dim & 7) * 2;
      *reinterpret_cast<bf16x4 *>(dst) = o;
    }
  }
  // fc weights of this head's K half for this wave's two column blocks (32 VGPRs), in flight during attention
  const rsrc_t wf = rsrc(p.wfc, (uint32_t)D * D * 2u);
  bf16x8 fw[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int nb = 2 * w + i;
      fw[s][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                wf, (uint32_t)lane * 16u + (uint32_t)(nb & 3) * 1024u,
                                                (uint32_t)(((nb >> 2) * (D / 32) + 4 * hh + s) * kUnit), 0));
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();

  // ---- head hh's attention: waves 0..3, queries 16 w + li
  f32x4 oacc[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float l_run = 0.f;
  if (w < 4 && len > 0) {
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[s] = *reinterpret_cast<const bf16x8 *>(smem + Q_OFF + (16 * w + li) * QP + (32 * s + 8 * g) * 2);
    const char *Kb = smem + K_OFF;
    const char *Vb = smem + V_OFF;
    constexpr int NBK = LMAX / 16;
    f32x4 sacc[NBK];
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni) {
      sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(Kb + kv_off(ni * 16 + li, 4 * s + g));
        sacc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sacc[ni], 0, 0, 0);
      }
    }
    const int lim = len - 4 * g;
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ni * 16 + j >= lim) sacc[ni][j] = -INFINITY;
    float mx = -INFINITY;
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni) {
      mx = max_nn(max_nn(mx, sacc[ni][0]), sacc[ni][1]);
      mx = max_nn(max_nn(mx, sacc[ni][2]), sacc[ni][3]);
    }
    const float m_new = rows_max(mx);
    const float mc = -m_new * p.scale_log2;
    float sx = 0.f, sy = 0.f;
    bf16x8 pf[NBK / 2];
#pragma unroll
    for (int ni = 0; ni < NBK; ++ni)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const float px = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp], p.scale_log2, mc));
        const float py = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ni][2 * jp + 1], p.scale_log2, mc));
        sx += px;
        sy += py;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp] = (bf16)px;
        pf[ni >> 1][(ni & 1) * 4 + 2 * jp + 1] = (bf16)py;
      }
    l_run = rows_sum(sx + sy);
    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int s2 = 0; s2 < NBK / 2; ++s2) {
#pragma unroll
      for (int h4 = 0; h4 < DK / 64; ++h4) {
        bf16x8 vf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int nd = 4 * h4 + i;
          const char *vp = Vb + kv_off(4 * g + tq, nd * 2 + (tp >> 1)) + (tp & 1) * 8 + s2 * 32 * 256;
          auto lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)vp);
          auto hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(vp + 16 * 256));
          __builtin_memcpy(&vf[i], &lo, 8);
          __builtin_memcpy(reinterpret_cast<char *>(&vf[i]) + 8, &hi, 8);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          oacc[4 * h4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[i], pf[s2], oacc[4 * h4 + i], 0, 0, 0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();  // the Q fragments are read: the Q region becomes o_h [64][QP]
  if (w < 4) {
    const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
    const int q = 16 * w + li;
#pragma unroll
    for (int nd = 0; nd < DK / 16; ++nd) {
      const bf16x4 o = {(bf16)(oacc[nd][0] * inv), (bf16)(oacc[nd][1] * inv), (bf16)(oacc[nd][2] * inv),
                        (bf16)(oacc[nd][3] * inv)};
      *reinterpret_cast<bf16x4 *>(smem + Q_OFF + q * QP + (nd * 16 + 4 * g) * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();

  // ---- fc_h: columns 32 w .. 32 w + 31 over K = this head's 128 dims
  f32x4 fa[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) fa[i][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 of[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      of[mb] = *reinterpret_cast<const bf16x8 *>(smem + Q_OFF + (16 * mb + li) * QP + s * 64 + g * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) fa[i][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s][i], of[mb], fa[i][mb], 0, 0, 0);
  }
  // ---- hand-off: partial rows through the workspace (sc1 both ways), the last arriver finishes
  const rsrc_t pr = rsrc(p.part, p.part_bytes);
  auto pofs = [&](int head, int i, int mb) {
    return (uint32_t)(b * 2 + head) * 65536u + (uint32_t)((((w * 2 + i) * 4 + mb) * 64 + lane) * 16);
  };
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, fa[i][mb]),
                                             pr, pofs(hh, i, mb), 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  int *flag = reinterpret_cast<int *>(smem + RED_OFF);
  if (tid == 0) {
    // acq_rel: the partner's sc1 partial stores are ordered before its add, ours after
    const int old = __hip_atomic_fetch_add(p.cnt + b, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == 1;
    if (last) __hip_atomic_store(p.cnt + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for the next launch
    *flag = last;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();
  if (!*flag) return;
  bar();  // every wave read the flag before the reduction reuses the slot
  {
    f32x4 other[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        other[i][mb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, pofs(hh ^ 1, i, mb), 0, 16));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) fa[i][mb] = hh == 0 ? fa[i][mb] + other[i][mb] : other[i][mb] + fa[i][mb];
  }
  // + bfc + x, LayerNorm over the 8 waves, row mask, staged whole-row stores (as the one-workgroup form)
  float *red = reinterpret_cast<float *>(smem + RED_OFF);
  float part[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = 16 * mb + li;
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = 16 * (2 * w + i) + 4 * g;
      const float4 bb = *reinterpret_cast<const float4 *>(vfc + n);
      const bf16x4 xv = *reinterpret_cast<const bf16x4 *>(smem + X_OFF + m * XP + n * 2);
      f32x4 v = fa[i][mb];
      v[0] = v[0] + bb.x + (float)xv[0];
      v[1] = v[1] + bb.y + (float)xv[1];
      v[2] = v[2] + bb.z + (float)xv[2];
      v[3] = v[3] + bb.w + (float)xv[3];
      fa[i][mb] = v;
      sm += (v[0] + v[1]) + (v[2] + v[3]);
    }
    part[mb] = rows_sum(sm);
  }
  // across the 8 waves through LDS; the two passes use separate slots (one barrier each)
  auto reduce = [&](float (&pv)[4], float (&tot)[4], int pass) {
    float *rb = red + pass * LMAX * 8;
    if (g == 0) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) rb[(16 * mb + li) * 8 + w] = pv[mb];
    }
    bar();
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const float4 a = *reinterpret_cast<const float4 *>(rb + (16 * mb + li) * 8);
      const float4 c = *reinterpret_cast<const float4 *>(rb + (16 * mb + li) * 8 + 4);
      tot[mb] = ((a.x + a.y) + (a.z + a.w)) + ((c.x + c.y) + (c.z + c.w));
    }
  };
  float mean[4], var[4];
  reduce(part, mean, 0);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    mean[mb] *= 1.0f / D;
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 d = fa[i][mb];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] -= mean[mb];
      fa[i][mb] = d;
      sm += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
    }
    part[mb] = rows_sum(sm);
  }
  reduce(part, var, 1);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = 16 * mb + li;
    const float rstd = 1.0f / sqrtf(var[mb] * (1.0f / D) + p.eps);
    const float keep = m < len ? 1.0f : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = 16 * (2 * w + i) + 4 * g;
      const float4 gg = *reinterpret_cast<const float4 *>(vg + n);
      const float4 be = *reinterpret_cast<const float4 *>(vb + n);
      const f32x4 d = fa[i][mb];
      const bf16x4 o = {(bf16)((d[0] * rstd * gg.x + be.x) * keep), (bf16)((d[1] * rstd * gg.y + be.y) * keep),
                        (bf16)((d[2] * rstd * gg.z + be.z) * keep), (bf16)((d[3] * rstd * gg.w + be.w) * keep)};
      *reinterpret_cast<bf16x4 *>(smem + X_OFF + m * XP + n * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  bar();
  uint4 *orow = reinterpret_cast<uint4 *>(p.out + (size_t)xrow0 * D);
  for (int i = tid; i < L * (D * 2 / 16); i += NT) {
    const int m = i >> 5, c = i & 31;
    orow[i] = *reinterpret_cast<const uint4 *>(smem + X_OFF + m * XP + c * 16);
  }
}

}  // namespace

static int enc_block_launch(const void *x, const int64_t *tokens, const float *emb, int vocab, const float *pe,
                            int32_t *bad_ids, const int64_t *lens, int B, int L, const void *wqkv, const float *bqkv,
                            const void *wfc, const float *bfc, const float *gamma, const float *beta, float eps, int H,
                            int dk, float temperature, void *out, uint8_t *src_mask, const int64_t *mel_lens, int T_mel,
                            uint8_t *mel_mask, const fs2_cond_desc *cond, void *ws, int64_t ws_bytes,
                            fs2_stream_t stream) {
  const bool embed = tokens != nullptr;
  if ((!embed && x == nullptr) || (embed && (emb == nullptr || pe == nullptr || vocab <= 0)) || lens == nullptr ||
      wqkv == nullptr || bqkv == nullptr || wfc == nullptr || bfc == nullptr || gamma == nullptr || beta == nullptr ||
      out == nullptr || !(temperature > 0.f))
    return FS2_EINVAL;
  if (B < 0 || L < 0 || (mel_mask != nullptr && (mel_lens == nullptr || T_mel < 0))) return FS2_EINVAL;
  if (H != 2 || dk != DK || L > LMAX) return FS2_EUNSUPPORTED;
  if (x == out) return FS2_EINVAL;
  if (B == 0 || L == 0) return FS2_OK;
  if ((int64_t)B * L * D * 2 >= (1LL << 31)) return FS2_EUNSUPPORTED;
  EncBlockArgs a{};
  a.x = reinterpret_cast<const bf16 *>(x);
  a.lens = lens;
  a.B = B;
  a.L = L;
  a.wqkv = reinterpret_cast<const bf16 *>(wqkv);
  a.bqkv = bqkv;
  a.wfc = reinterpret_cast<const bf16 *>(wfc);
  a.bfc = bfc;
  a.gamma = gamma;
  a.beta = beta;
  a.eps = eps;
  a.scale_log2 = 1.4426950408889634f / temperature;
  a.out = reinterpret_cast<bf16 *>(out);
  a.tokens = tokens;
  a.emb = emb;
  a.pe = pe;
  a.vocab = vocab;
  a.bad = bad_ids;
  a.src_mask = src_mask;
  a.mel_lens = mel_lens;
  a.T_mel = T_mel;
  a.mel_mask = mel_mask;
  // the head-split form when a workspace is given (2 workgroups per utterance, sc1 hand-off)
  a.cnt = reinterpret_cast<int *>(ws);
  a.part = ws != nullptr ? static_cast<char *>(ws) + 4096 : nullptr;
  a.part_bytes = (uint32_t)(ws_bytes > 4096 ? ws_bytes - 4096 : 0);
  a.ncond = a.ncx = 0;
  if (cond != nullptr && (cond->speaker_table != nullptr || cond->emo_table != nullptr)) {
    if (!embed) return FS2_EINVAL;
    if (cond->speaker_table != nullptr && (cond->speakers == nullptr || cond->spk_out == nullptr || cond->n_speaker <= 0))
      return FS2_EINVAL;
    if (cond->emo_table != nullptr &&
        (cond->emotions == nullptr || cond->arousals == nullptr || cond->valences == nullptr || cond->aro_table == nullptr ||
         cond->val_table == nullptr || cond->lin_w == nullptr || cond->lin_b == nullptr || cond->emo_out == nullptr ||
         cond->n_emo <= 0 || cond->n_aro <= 0 || cond->n_val <= 0))
      return FS2_EINVAL;
    const int dc = cond->emo_table != nullptr ? cond->d_emo + cond->d_aro + cond->d_val : 0;
    if ((int64_t)kCondU * (dc + 256) * 4 > SMEM) return FS2_EUNSUPPORTED;
    a.cond = CondArgs{cond->speakers, cond->speaker_table, cond->n_speaker, cond->emotions, cond->emo_table, cond->n_emo,
                      cond->d_emo, cond->arousals, cond->aro_table, cond->n_aro, cond->d_aro, cond->valences,
                      cond->val_table, cond->n_val, cond->d_val, cond->lin_w, cond->lin_b, B, D, cond->spk_out,
                      cond->emo_out};
    a.ncx = D / 64;
    a.ncond = a.ncx * ((B + kCondU - 1) / kCondU);
  }
  // the head-split form has no conditioning role: the one-workgroup form then
  const bool half = !ENC_TRACE && a.ncond == 0 && ws != nullptr && B <= 1024 &&
                    (int64_t)B * 2 * 65536 + 4096 <= ws_bytes;
  const unsigned nhalf = (unsigned)(((B + 7) / 8) * 16);
  if (half && embed)
    hipLaunchKernelGGL(enc_attn_half_kernel<true>, dim3(nhalf), dim3(NT), 0, as_stream(stream), a);
  else if (half)
    hipLaunchKernelGGL(enc_attn_half_kernel<false>, dim3(nhalf), dim3(NT), 0, as_stream(stream), a);
  else if (embed && a.ncond > 0)
    hipLaunchKernelGGL((enc_attn_block_kernel<true, true>), dim3((unsigned)(B + a.ncond)), dim3(NT), 0,
                       as_stream(stream), a);
  else if (embed)
    hipLaunchKernelGGL(enc_attn_block_kernel<true>, dim3((unsigned)B), dim3(NT), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(enc_attn_block_kernel<false>, dim3((unsigned)B), dim3(NT), 0, as_stream(stream), a);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_enc_attn_block(const void *x, const int64_t *lens, int B, int L, const void *wqkv, const float *bqkv,
                                  const void *wfc, const float *bfc, const float *gamma, const float *beta, float eps,
                                  int H, int dk, float temperature, void *out, void *ws, int64_t ws_bytes,
                                  fs2_stream_t stream) {
  return enc_block_launch(x, nullptr, nullptr, 0, nullptr, nullptr, lens, B, L, wqkv, bqkv, wfc, bfc, gamma, beta, eps, H,
                          dk, temperature, out, nullptr, nullptr, 0, nullptr, nullptr, ws, ws_bytes, stream);
}

extern "C" int fs2_enc_embed_attn_block(const int64_t *tokens, const float *emb, int vocab, const float *pe,
                                        int32_t *bad_ids, const int64_t *lens, int B, int L, const void *wqkv,
                                        const float *bqkv, const void *wfc, const float *bfc, const float *gamma,
                                        const float *beta, float eps, int H, int dk, float temperature, void *out,
                                        uint8_t *src_mask, const int64_t *mel_lens, int T_mel, uint8_t *mel_mask,
                                        const fs2_cond_desc *cond, void *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (tokens == nullptr) return FS2_EINVAL;
  return enc_block_launch(nullptr, tokens, emb, vocab, pe, bad_ids, lens, B, L, wqkv, bqkv, wfc, bfc, gamma, beta, eps,
                          H, dk, temperature, out, src_mask, mel_lens, T_mel, mel_mask, cond, ws, ws_bytes, stream);
}
