// PositionwiseFeedForward + residual + LayerNorm for SMALL row counts (the encoder's B x L_max
// phoneme rows, a free-running decoder's ~10k frames) as two wide-tile launches:
//
//   launch 1 (ffn_hidden_kernel): H = relu(Conv1d_k9(x; w1) + b1)        [rows, F] bf16
//   launch 2 (ffn_out_kernel):    y = LN(H . w2^T + b2 + x) ; masked ; (+ addvecs)
//                                                        -- transformer/SubLayers.py:85-93
//
// Why: the fused kernel (ffn.hip) streams ALL 5.2 MB of FFN weights through every workgroup, which is
// right when 112-row tiles fill the chip (the cfg2 decoder's 24.9k frames) but not at 4k rows: there
// it needs 64-row tiles split 4 ways over the hidden dimension, each workgroup pulling 1.3 MB of
// weights for 64 rows at the ~70 GB/s an XCD's L2 delivers per CU (MI355X_MICROARCH.md, L2 table),
// plus a 196 KB partial hand-off: 39-42 us per encoder block at 0.21 of the MFMA peak.
//
// Launch 1 tiles 256 rows x 64 hidden columns (cfg2 encoder: 16 x 16 = 256 workgroups, one per CU):
// the x tile (256 + KS - 1 rows, all 256 channels, 144 KB) stays in LDS for all 9 taps and the
// workgroup streams only its 64-column slice of w1 (288 KB): ~0.44 MB per CU instead of ~1.5 MB. 4
// waves = 2 row halves x 2 hidden halves: a wave's k-step is 2 weight fragments (its 32 hidden rows,
// from the ffn.hip fragment-ordered image, through a register ring 8 k-steps deep), 8 B fragments
// from the x tile and 16 MFMAs; the B fragments of one row half are shared through L1-free LDS reads
// (32 KB of LDS reads and 8 KB of L1 weight reads per k-step per CU: half of either unit's rate).
//
// Launch 2 tiles 64 rows x 64 output columns (4 column quarters per row tile): K = F split over the
// 4 waves (every load of the workgroup -- 128 KB of w2, 128 KB of H -- issued at once: one memory
// round trip), the 4 partials summed in wave order through LDS, + b2 + the residual; the LayerNorm
// needs whole 256-column rows, so each quarter stores its f32 pre-norm rows (write-through) into the
// split-K workspace, and the last of the 4 to arrive (an arrival counter per row tile, as ffn.hip's
// split-hidden form) normalises all 256 columns of the tile's rows: mask, addvecs, bf16 out.
//
// Both GEMMs accumulate in the fused kernel's k order (k-steps of 32 channels, tap-major for w1,
// hidden order for w2), so H and the pre-norm sums are the fused kernel's; only the LayerNorm's row
// statistics are summed in a different order (tests/test_gpu_ffn.py: within bf16 rounding).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

constexpr int kWD = 256;          // d_model
constexpr int kWUnit = 4096;      // ffn.hip weight unit: 64 rows x 32 channels, fragment order
constexpr int kWLgkm0 = 0xC07F;

template <int N, typename Fn, int... I>
__device__ __forceinline__ void wfor_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void wfor(Fn &&f) {
  wfor_impl<N>(f, std::make_integer_sequence<int, N>{});
}

struct WideArgs {
  const bf16 *x;         // FFN input rows (also the residual), row stride xs elements
  int64_t xs;
  uint32_t x_bytes;
  const bf16 *w;         // ffn.hip fragment-ordered w1 | w2 (ops.pack_ffn_weights)
  uint32_t w_bytes;
  const float *b1, *b2, *gamma, *beta;
  float eps;
  const int64_t *lens;   // padded rows: [B] lengths (mask), else null
  const float *av1, *av2;  // padded rows: [B, 256] vectors added after the mask, or null
  const int *rows_dev;   // packed rows: device row count, else null
  const int2 *row_pos;   // packed rows: (position, length) per row
  int M, T, pad, F;
  bf16 *h;               // [M, F] hidden
  uint32_t h_bytes;
  int *cnt;              // [row tiles] arrival counters (zero between launches)
  float *z;              // [M, 256] f32 pre-norm rows (split-K workspace)
  uint32_t z_bytes;
  bf16 *out;
  int64_t os;
  int nslices, ntiles;   // launch 1: hidden slices (F / 64) and 256-row tiles; launch 2: 64-row tiles
};

// ---------------------------------------------------------------------------------------------------
// launch 1: H = relu(conv_k(x) + b1) on 256-row x 64-column tiles
template <int KS>
__global__ __launch_bounds__(256, 1) void ffn_hidden_kernel(WideArgs p) {
  constexpr int BM = 256, XROWS = BM + KS - 1, XPITCH = 544;
  constexpr int XPIECES = (XROWS * XPITCH + 1023) / 1024, XP_PER_WAVE = (XPIECES + 3) / 4;
  constexpr int X_OFF = 512;  // [0, 512): zeros, the masked tap rows' fragment source
  constexpr int SMEM = X_OFF + 4 * XP_PER_WAVE * 1024;
  static_assert(SMEM <= 163840, "LDS");
  static_assert(BM * 144 <= 4 * XP_PER_WAVE * 1024, "H staging fits in the x region");
  constexpr int NK = KS * (kWD / 32);  // k-steps (tap-major, 8 per tap)
  constexpr int DEPTH = 8;             // weight k-steps in flight per wave (one tap ahead)
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rh = w & 1, hh = w >> 1;  // row half (128 rows), hidden half (32 columns) of the tile
  // XCD-aware order: consecutive L run on one XCD (blockIdx.x & 7 picks the XCD), slice-major, so an
  // XCD holds ~2 hidden slices' weights and all the x rows in its L2
  const int L = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int slice = L / p.ntiles, tile = L - slice * p.ntiles;
  if (slice >= p.nslices) return;
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M;
  const int m0 = tile * BM;
  if (m0 >= M) return;
  const int pad = p.pad, T = p.T;

  // the zero region first: a ds_write behind the tile's LDS-DMA would wait for all of it
  if (tid < 32) *reinterpret_cast<float4 *>(smem + 16 * tid) = make_float4(0.f, 0.f, 0.f, 0.f);
  // x tile (rows m0 - pad .. m0 + BM + KS - 2) -> LDS by LDS-DMA, lane-linear 1 KiB pieces
  {
    const rsrc_t sr = make_rsrc(p.x, p.x_bytes);
    const uint32_t srow = (uint32_t)p.xs * 2u;
#pragma unroll
    for (int i = 0; i < XP_PER_WAVE; ++i) {
      const int pc = w + 4 * i;
      const int o = pc * 1024 + lane * 16;
      const int r = o / XPITCH, within = o - r * XPITCH;
      const int gm = m0 - pad + r;
      const bool ok = r < XROWS && within < 512 && gm >= 0 && gm < M;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(sr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                               16, ok ? (uint32_t)gm * srow + (uint32_t)within : kOOB, 0, 0, 0);
    }
  }

  // row positions of this lane's 8 row blocks and b1 of its 8 hidden columns: loads issued here,
  // used after the weight ring starts (one wait covers them with the x tile)
  constexpr int MB = 8;
  // (padded rows: position m % T of a length-T sequence, computed first; packed rows: loaded over
  // them -- ALU writes after the loads into the same registers would wait for the loads)
  int2 rq[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = min(m0 + rh * 128 + mb * 16 + (lane & 15), M - 1);
    rq[mb] = make_int2(m % T, T);
  }
  if (p.row_pos != nullptr) {  // uniform branch around the whole loop: no wait between the loads
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) rq[mb] = p.row_pos[min(m0 + rh * 128 + mb * 16 + (lane & 15), M - 1)];
  }
  const int hcol0 = slice * 64 + hh * 32 + 4 * (lane >> 4);
  const float4 bb0 = *reinterpret_cast<const float4 *>(p.b1 + hcol0);
  const float4 bb1 = *reinterpret_cast<const float4 *>(p.b1 + hcol0 + 16);

  // weight ring: unit k of this slice at (slice * NK + k) * 4 KiB; this wave's two 1 KiB fragments
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t wbase = (uint32_t)(slice * NK) * (uint32_t)kWUnit + (uint32_t)(hh * 2048 + lane * 16);
  bf16x8 pa[DEPTH][2];
  auto load_at = [&](auto S, int k) {
    constexpr int s = decltype(S)::value;
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t o = wbase + (uint32_t)min(k, NK - 1) * (uint32_t)kWUnit;
    pa[s][0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, o, 0, 0));
    pa[s][1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, o + 1024, 0, 0));
    __builtin_amdgcn_sched_barrier(0);
  };
  wfor<DEPTH>([&](auto I) { load_at(I, decltype(I)::value); });
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DEPTH) : "memory");  // x tile, rows, b1 (older than the ring)
  // tap validity per row block: bit tap set when row + tap - pad stays inside its sequence
  int vmask[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    int v = 0;
#pragma unroll
    for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(rq[mb].x + tap - pad) < (unsigned)rq[mb].y ? 1 : 0) << tap;
    vmask[mb] = v;
  }
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  const int hrow0 = rh * 128 + (lane & 15), hi = lane >> 4;
  auto bases = [&](int tap, int (&ad)[MB]) {
    const int base = X_OFF + (hrow0 + tap) * XPITCH + hi * 16;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) ad[mb] = (base + mb * 16 * XPITCH) & __builtin_amdgcn_sbfe(vmask[mb], tap, 1);
  };
  auto issue = [&](const int (&ad)[MB], auto KSI, bf16x8 (&f)[MB]) {
    constexpr int off = decltype(KSI)::value * 64;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) f[mb] = *reinterpret_cast<const bf16x8 *>(smem + ad[mb] + off);
  };
  f32x4 acc[2][MB];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&fa)[2], const bf16x8 (&fb)[MB]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[jb], fb[mb], acc[jb][mb], 0, 0, 0);
  };
  bf16x8 f0[MB], f1[MB];
  int bc[MB], bn[MB];
  bases(0, bc);
  issue(bc, std::integral_constant<int, 0>{}, f0);
#pragma nounroll
  for (int tap = 0; tap < KS; ++tap) {
    bases(tap + 1, bn);  // tap KS: every row masked (the zero region): harmless reads
    wfor<8>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value;
      if constexpr (ks + 1 < 8) {
        if constexpr (ks & 1)
          issue(bc, std::integral_constant<int, ks + 1>{}, f0);
        else
          issue(bc, std::integral_constant<int, ks + 1>{}, f1);
      } else {
        issue(bn, std::integral_constant<int, 0>{}, f0);
      }
      if constexpr (ks & 1)
        mma(pa[ks], f1);
      else
        mma(pa[ks], f0);
      load_at(std::integral_constant<int, ks>{}, (tap + 1) * 8 + ks);  // past the end: unit NK - 1 again
    });
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) bc[mb] = bn[mb];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __builtin_amdgcn_s_barrier();  // every wave done with the x tile: stage H over it

  // H = bf16(relu(acc + b1)): lane holds hidden columns 4 hi .. +3 of block jb, row hrow0 + 16 mb;
  // staged at a 144-byte row pitch, then whole 128-byte row segments out (8 x 16 B per row)
  constexpr int HP = 144;
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const float4 bb = jb == 0 ? bb0 : bb1;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[jb][mb];
      bf16x4 o;
      o[0] = (bf16)fmaxf(v[0] + bb.x, 0.f);
      o[1] = (bf16)fmaxf(v[1] + bb.y, 0.f);
      o[2] = (bf16)fmaxf(v[2] + bb.z, 0.f);
      o[3] = (bf16)fmaxf(v[3] + bb.w, 0.f);
      *reinterpret_cast<bf16x4 *>(smem + X_OFF + (hrow0 + 16 * mb) * HP + (hh * 32 + jb * 16 + 4 * hi) * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __syncthreads();
  const uint32_t hrow = (uint32_t)p.F * 2u;
  char *hb = reinterpret_cast<char *>(p.h);
#pragma unroll
  for (int i = 0; i < BM * 8 / 256; ++i) {
    const int e = tid + 256 * i, r = e >> 3, c = e & 7;
    if (m0 + r < M)
      *reinterpret_cast<uint4 *>(hb + (uint32_t)(m0 + r) * hrow + (uint32_t)(slice * 128 + c * 16)) =
          *reinterpret_cast<const uint4 *>(smem + X_OFF + r * HP + c * 16);
  }
}

// ---------------------------------------------------------------------------------------------------
// launch 2: z = H . w2^T + b2 + x on 64-row x 64-column tiles, then the LayerNorm by the last of the
// row tile's 4 column quarters
template <int F>
__global__ __launch_bounds__(256, 1) void ffn_out_kernel(WideArgs p) {
  constexpr int NK = F / 32;       // k-steps of 32 hidden columns
  constexpr int KW = NK / 4;       // per wave
  constexpr int RED = 4 * 16 * 64 * 16;  // 4 waves' partial tiles in LDS: [wave][jb * 4 + mb][lane] f32x4
  __shared__ __attribute__((aligned(16))) char smem[RED + 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the 4 quarters of a row tile adjacent in L (one XCD: the hand-off stays in its L2)
  const int L = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int tile = L >> 2, q = L & 3;
  if (tile >= p.ntiles) return;
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M;
  const int m0 = tile * 64;
  if (m0 >= M) return;
  const int T = p.T;
  const int hi = lane >> 4, r16 = lane & 15;

  // every operand of this wave's K quarter at once: KW k-steps x (4 w2 fragments + 4 H fragments)
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const rsrc_t hr = make_rsrc(p.h, p.h_bytes);
  bf16x8 wa[KW][4], hb[KW][4];
  // w2 units after w1 (the last kWD * F elements of the image): quarter q's k-step kk at unit q * NK + kk
  const uint32_t wb = p.w_bytes - (uint32_t)(kWD * F * 2) + (uint32_t)((q * NK + w * KW) * kWUnit) + (uint32_t)lane * 16u;
  const uint32_t hrow = (uint32_t)F * 2u;
#pragma unroll
  for (int k = 0; k < KW; ++k) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
      wa[k][jb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, wb + k * kWUnit + jb * 1024, 0, 0));
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m = m0 + mb * 16 + r16;
      hb[k][mb] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      hr, m < M ? (uint32_t)m * hrow + (uint32_t)((w * KW + k) * 64 + hi * 16) : kOOB, 0, 0));
    }
  }
  // all loads stay ahead of the MFMAs (left alone, hipcc interleaves them to save registers and
  // every k-step then waits for its own memory round trip)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[4][4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KW; ++k)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[k][jb], hb[k][mb], acc[jb][mb], 0, 0, 0);
  // the 4 K-quarter partials through LDS, summed in wave order by the wave owning row block mb = w
  f32x4 *red = reinterpret_cast<f32x4 *>(smem);
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) red[(w * 16 + jb * 4 + mb) * 64 + lane] = acc[jb][mb];
  __syncthreads();
  f32x4 zv[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    f32x4 s = red[(0 * 16 + jb * 4 + w) * 64 + lane];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) s += red[(ww * 16 + jb * 4 + w) * 64 + lane];
    zv[jb] = s;
  }
  // + b2 + residual; lane: row m0 + 16 w + r16, columns 64 q + 16 jb + 4 hi .. + 3
  const int m = m0 + 16 * w + r16;
  const bool mok = m < M;
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const rsrc_t zr = make_rsrc(p.z, p.z_bytes);
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int n = 64 * q + 16 * jb + 4 * hi;
    const float4 b2 = *reinterpret_cast<const float4 *>(p.b2 + n);
    const uint2 xv = bload8(xr, mok ? (uint32_t)m * (uint32_t)p.xs * 2u + (uint32_t)n * 2u : kOOB);
    const bf16x4 x4 = __builtin_bit_cast(bf16x4, xv);
    f32x4 v = zv[jb];
    v[0] = v[0] + b2.x + (float)x4[0];
    v[1] = v[1] + b2.y + (float)x4[1];
    v[2] = v[2] + b2.z + (float)x4[2];
    v[3] = v[3] + b2.w + (float)x4[3];
    // write-through (sc1): the last-arriving quarter reads it with sc1 loads from another CU
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), zr,
                                           mok ? ((uint32_t)m * kWD + (uint32_t)n) * 4u : kOOB, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int *flag = reinterpret_cast<int *>(smem + RED);
  if (tid == 0) {
    // relaxed add + sc1 stores / loads of every handed-off byte, each storing wave drained before the
    // barrier ahead of this add, one workgroup per CU: ffn.hip's split-hidden hand-off
    const int old = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == 3;
    if (last) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;

  // LayerNorm of the tile's rows over all 256 columns: wave w takes rows 16 w + r16; lane (r16, hi)
  // holds columns 16 i + 4 hi .. + 3, i = 0..15 (64 values); row sums over the 4 lanes of a row
  f32x4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         zr, mok ? ((uint32_t)m * kWD + (uint32_t)(16 * i + 4 * hi)) * 4u : kOOB, 0, 16));
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mean = s * (1.0f / 256.0f);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] -= mean;
    ss += (v[i][0] * v[i][0] + v[i][1] * v[i][1]) + (v[i][2] * v[i][2] + v[i][3] * v[i][3]);
  }
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  const float rstd = 1.0f / sqrtf(ss * (1.0f / 256.0f) + p.eps);
  bool masked = false;
  int bb = 0;
  if (p.row_pos == nullptr && mok) {
    bb = m / T;
    masked = p.lens != nullptr && (int64_t)(m - bb * T) >= p.lens[bb];
  }
  if (!mok) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = 16 * i + 4 * hi;
    const float4 g = *reinterpret_cast<const float4 *>(p.gamma + n);
    const float4 be = *reinterpret_cast<const float4 *>(p.beta + n);
    float y[4] = {v[i][0] * rstd * g.x + be.x, v[i][1] * rstd * g.y + be.y, v[i][2] * rstd * g.z + be.z,
                  v[i][3] * rstd * g.w + be.w};
    if (masked) y[0] = y[1] = y[2] = y[3] = 0.f;
    if (p.av1 != nullptr) {
      const float4 a1 = *reinterpret_cast<const float4 *>(p.av1 + (int64_t)bb * kWD + n);
      y[0] += a1.x; y[1] += a1.y; y[2] += a1.z; y[3] += a1.w;
    }
    if (p.av2 != nullptr) {
      const float4 a2 = *reinterpret_cast<const float4 *>(p.av2 + (int64_t)bb * kWD + n);
      y[0] += a2.x; y[1] += a2.y; y[2] += a2.z; y[3] += a2.w;
    }
    bf16x4 o;
    o[0] = (bf16)y[0];
    o[1] = (bf16)y[1];
    o[2] = (bf16)y[2];
    o[3] = (bf16)y[3];
    *reinterpret_cast<bf16x4 *>(p.out + (int64_t)m * p.os + n) = o;
  }
}

}  // namespace

extern "C" int fs2_ffn_wide(const fs2_ffn_desc *d, void *hidden, int64_t hidden_bytes, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->b1 == nullptr || d->b2 == nullptr ||
      d->ln_gamma == nullptr || d->ln_beta == nullptr || d->out == nullptr || hidden == nullptr)
    return FS2_EINVAL;
  if (d->B < 0 || d->T < 0 || d->x_row_stride < kWD || (d->x_row_stride & 7) || d->out_row_stride < kWD ||
      (d->out_row_stride & 7))
    return FS2_EINVAL;
  if (d->D != kWD || !(d->F == 1024 || d->F == 512) || !(d->KS == 9 || d->KS == 3) || d->pad < 0 ||
      d->pad > d->KS - 1)
    return FS2_EUNSUPPORTED;
  if (d->wqkv != nullptr || d->pre_att != nullptr) return FS2_EUNSUPPORTED;  // fused-kernel extras
  if ((d->rows_dev == nullptr) != (d->row_pos == nullptr)) return FS2_EINVAL;
  if (d->rows_dev != nullptr && (d->lens != nullptr || d->addvec1 != nullptr || d->addvec2 != nullptr))
    return FS2_EINVAL;
  if (d->x == d->out || hidden == d->x || hidden == d->out) return FS2_EINVAL;
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 > 0x7fffff00LL || d->rows_max < 0) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;
  const int64_t Mg = (d->rows_dev != nullptr && d->rows_max > 0 && d->rows_max < M64) ? d->rows_max : M64;
  const int64_t xb = M64 * d->x_row_stride * 2;
  const int64_t wb = ((int64_t)d->F * d->KS * kWD + (int64_t)kWD * d->F) * 2;  // ffn.hip: w1 | w2
  const int64_t hb = Mg * d->F * 2;
  const int ntiles64 = (int)((Mg + 63) / 64);
  const int64_t zb = Mg * kWD * 4;
  if (xb >= (1LL << 31) || hb >= (1LL << 31) || hidden_bytes < hb) return FS2_EUNSUPPORTED;
  if (d->splitk_ws == nullptr || ntiles64 > 1024 || d->splitk_ws_bytes < 4096 + zb || zb >= (1LL << 31))
    return FS2_EINVAL;
  WideArgs p{};
  p.x = reinterpret_cast<const bf16 *>(d->x);
  p.xs = d->x_row_stride;
  p.x_bytes = (uint32_t)xb;
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.w_bytes = (uint32_t)wb;
  p.b1 = d->b1;
  p.b2 = d->b2;
  p.gamma = d->ln_gamma;
  p.beta = d->ln_beta;
  p.eps = d->ln_eps;
  p.lens = d->lens;
  p.av1 = d->addvec1;
  p.av2 = d->addvec2;
  p.rows_dev = d->rows_dev;
  p.row_pos = reinterpret_cast<const int2 *>(d->row_pos);
  p.M = (int)Mg;
  p.T = d->T;
  p.pad = d->pad;
  p.F = d->F;
  p.h = static_cast<bf16 *>(hidden);
  p.h_bytes = (uint32_t)hb;
  p.cnt = static_cast<int *>(d->splitk_ws);
  p.z = reinterpret_cast<float *>(static_cast<char *>(d->splitk_ws) + 4096);
  p.z_bytes = (uint32_t)zb;
  p.out = static_cast<bf16 *>(d->out);
  p.os = d->out_row_stride;
  hipStream_t s = as_stream(stream);
  // launch 1: hidden slices x 256-row tiles, grid padded to whole XCD rounds
  p.nslices = d->F / 64;
  p.ntiles = (int)((Mg + 255) / 256);
  const int n1 = (p.nslices * p.ntiles + 7) & ~7;
  if (d->KS == 9)
    hipLaunchKernelGGL((ffn_hidden_kernel<9>), dim3(n1), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((ffn_hidden_kernel<3>), dim3(n1), dim3(256), 0, s, p);
  FS2_CHECK_LAUNCH();
  // launch 2: 64-row tiles x 4 column quarters
  p.ntiles = ntiles64;
  const int n2 = (ntiles64 * 4 + 7) & ~7;
  if (d->F == 1024)
    hipLaunchKernelGGL((ffn_out_kernel<1024>), dim3(n2), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((ffn_out_kernel<512>), dim3(n2), dim3(256), 0, s, p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
