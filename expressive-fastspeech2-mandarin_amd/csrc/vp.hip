// VariancePredictor row kernels of the column-split form (model/modules.py:197-250).
//
// A VariancePredictor is Conv1d(k=3) -> ReLU -> LayerNorm -> Conv1d(k=3) -> ReLU -> LayerNorm ->
// Linear(256 -> 1) -> masked_fill on M = B*L ~ 4k rows. As LayerNorm-epilogue GEMMs every
// workgroup needs whole 256-wide rows, i.e. streams the whole weight matrix from L2 (~70 GB/s
// per CU: 20+ us per conv for the bf16x3 weights, whatever the row tile). Here the two convs are
// plain fs2_conv1d launches whose workgroups own column slices (duration + pitch side by side,
// N = 512), and the two LayerNorms are these bandwidth kernels between them:
//   fs2_vp_norm  relu(conv1) f32 -> LayerNorm -> the bf16 hi / lo planes conv2 reads (bf16x3)
//   fs2_vp_head  relu(conv2) f32 -> LayerNorm -> dot(lin_w) + lin_b -> mask -> pred, and for one
//                group the pitch / energy bucketize + embedding add (modules.py:80-100,117-126)
// One half-wave per (row, group): 32 lanes x 8 columns, 16-byte loads and stores, DPP sums.
//
// fs2_vp_fused (round 4) replaces the whole chain for bf16 inputs: ONE launch per predictor set
// (duration + pitch, then energy), see vp_fused_kernel below.
#include <type_traits>
#include <utility>

#include <cstdlib>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

constexpr int kC = 256;  // filter_size: 32 lanes x 8 columns

__device__ __forceinline__ float hsum32(float v) {  // sum over the 32 lanes of a half-wave
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v + __shfl_xor(v, 16, 64);
}

// LayerNorm of 8 columns per lane (torch: biased variance, (x - mean) / sqrt(var + eps) * g + b;
// the same two-pass form as the LN epilogues of conv_gemm.hip)
__device__ __forceinline__ void ln8(float v[8], const float *gamma, const float *beta, int n, float eps) {
  float g8[8], b8[8];
  load8(gamma + n, g8);
  load8(beta + n, b8);
  float s1 = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s1 += v[q];
  const float mean = hsum32(s1) * (1.0f / kC);
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v[q] -= mean;
    ss += v[q] * v[q];
  }
  const float rstd = 1.0f / sqrtf(hsum32(ss) * (1.0f / kC) + eps);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] * rstd * g8[q] + b8[q];
}

__global__ __launch_bounds__(256) void vp_norm_kernel(const float *__restrict__ y, int64_t ys, int M, int G,
                                                      const float *__restrict__ gamma, const float *__restrict__ beta,
                                                      float eps, bf16 *__restrict__ out, int64_t os) {
  const int64_t item = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  if (item >= (int64_t)M * G) return;  // whole half-waves leave together
  const int64_t m = item / G;
  const int g = (int)(item - m * G);
  const int n = (threadIdx.x & 31) * 8;
  float v[8];
  load8(y + m * ys + g * kC + n, v);
  ln8(v, gamma + g * kC, beta + g * kC, n, eps);
  float hi[8], lo[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hi[q] = (float)(bf16)v[q];
    lo[q] = v[q] - hi[q];
  }
  bf16 *op = out + m * os + g * 2 * kC;
  store8(op + n, hi);
  store8(op + kC + n, lo);
}

template <typename TX>
__global__ __launch_bounds__(256) void vp_head_kernel(const float *__restrict__ y, int64_t ys, int T, int M, int G,
                                                      const float *__restrict__ gamma, const float *__restrict__ beta,
                                                      float eps, const float *__restrict__ lin_w,
                                                      const float *__restrict__ lin_b,
                                                      const int64_t *__restrict__ lens, float *__restrict__ pred,
                                                      int embed_g, TX *__restrict__ x, int64_t xs, int D,
                                                      const float *__restrict__ target, float control,
                                                      const float *__restrict__ bins, int nb,
                                                      const float *__restrict__ table) {
  const int64_t item = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  if (item >= (int64_t)M * G) return;
  const int64_t m = item / G;
  const int g = (int)(item - m * G);
  const int sub = threadIdx.x & 31, n = sub * 8;
  float v[8], w8[8];
  load8(y + m * ys + g * kC + n, v);
  ln8(v, gamma + g * kC, beta + g * kC, n, eps);
  load8(lin_w + g * kC + n, w8);
  float sd = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) sd += v[q] * w8[q];
  const float dot = hsum32(sd) + lin_b[g];
  const int64_t b = m / T, t = m - b * T;
  const float p = t >= lens[b] ? 0.0f : dot;
  if (g != embed_g) {
    if (sub == 0) pred[(int64_t)g * M + m] = p;
    return;
  }
  // pitch / energy embedding (fs2_variance_embed semantics): target given -> bucketize the target
  // and keep the prediction; otherwise the prediction is scaled by control first
  const float val = target != nullptr ? target[m] : p * control;
  if (sub == 0) pred[(int64_t)g * M + m] = target != nullptr ? p : val;
  int lo = 0, hi = nb;  // torch.bucketize(val, bins, right=False)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bins[mid] < val) lo = mid + 1; else hi = mid;
  }
  const float *trow = table + (int64_t)lo * D;
  TX *xrow = x + m * xs;
  for (int col = n; col < D; col += 256) {
    float a[8], e[8];
    load8(xrow + col, a);
    load8(trow + col, e);
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] += e[q];
    store8(xrow + col, a);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused VariancePredictor (model/modules.py:197-250) for bf16 inputs, split-precision bf16x3:
//
//   h  = LN1(relu(Conv1d_k3(x; w1) + b1))       x bf16 (x_lo = 0): x.w_hi + x.w_lo
//   y  = LN2(relu(Conv1d_k3(h; w2) + b2))       h = h_hi + h_lo:  h_hi.w_hi + h_hi.w_lo + h_lo.w_hi
//   p  = mask(y . lin_w + lin_b)                 (+ the pitch / energy bucketize + embedding add)
//
// One workgroup per (32-row tile of the flattened [B*L] rows, predictor g): conv1 runs on the 48
// rows m0-1 .. m0+46 (3 blocks of 16; the tile's rows and the one-row halo its conv2 taps read),
// the x tile (50 rows incl. conv1's halo) is DMA'd to LDS once, h stays in LDS as bf16 hi / lo
// planes, conv2's 32 rows end in the LN2 + dot epilogue. Nothing but the prediction (and for the
// embedding group x + table[bucket]) reaches HBM: the column-split form's 8 launches wrote and
// re-read 4 intermediates (f32 conv outputs, the hi / lo planes).
//
// As in ffn.hip the weights are the MFMA A operand and never touch LDS: wave w owns output
// channels 64w .. 64w+63 of both convs; a k-step (tap, 32 channels) is two 4 KiB units (w_hi,
// w_lo) in fragment order, streamed by fully coalesced 16-byte loads into a 4-k-step register ring;
// the whole per-wave stream (both convs) is one linear run of 96 units. Sequence boundaries (each
// utterance's L_max rows, zero padding beyond them: nn.Conv1d padding=1) are per-lane tap masks.
constexpr int kVpC = 256;
constexpr int kVpBM = 32;                 // output rows per workgroup
constexpr int kVpHR = 48;                 // conv1 rows: m0 - 1 .. m0 + 46
constexpr int kVpXR = 50;                 // x rows: m0 - 2 .. m0 + 47
constexpr int kVpPitch = 544;             // LDS row pitch (512 + 32): conflict-free b128 fragment reads
constexpr int kVpUnit = 4096;             // one wave unit: 4 blocks x 64 lanes x 16 B
constexpr int kVpKS = 24;                 // k-steps per conv: 3 taps x 8 channel steps
constexpr int kVpUnits = 2 * kVpKS * 2;   // per wave: 2 convs x 24 k-steps x (hi, lo)
constexpr uint32_t kVpWaveBytes = (uint32_t)kVpUnits * kVpUnit;
constexpr int kVpDepth = 4;               // k-steps in flight (8 units, 128 registers)
constexpr int kVpLgkm0 = 0xC07F;          // s_waitcnt lgkmcnt(0) as a real wait-count instruction
constexpr int kVpPrefetchMax = 24;        // warm-up loads per wave (x tile + ring + these <= 63 in flight):
                                          // the energy set's 16 workgroups per XCD cover the whole stream
constexpr int kVpScratchOff = 512 + 4 * ((((50 * 544 + 1023) / 1024) + 3) / 4) * 1024;  // = HHI_OFF

struct VpArgs {
  const bf16 *x;
  int64_t xs;
  uint32_t x_bytes, w_bytes;
  const bf16 *w;
  const float *vec;   // [G][7][256]
  const float *lin_b; // [G]
  float eps;
  int M, L, G, ntiles;
  const int64_t *lens;
  int prefetch;       // L2 warm-up of the weight stream (FS2_VP_PREFETCH, default on)
  float *pred;        // [G][M]
  int embed_g;
  bf16 *xo;
  int64_t xos;
  const float *target;
  float control;
  const float *bins;
  int nb;             // number of bin edges (n_bins - 1)
  const float *table; // [n_bins][256]
};

template <typename Fn, int... I>
__device__ __forceinline__ void vp_static_for_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void vp_static_for(Fn &&f) {
  vp_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__global__ __launch_bounds__(256, 1) void vp_fused_kernel(VpArgs p) {
  constexpr int XPIECES = (kVpXR * kVpPitch + 1023) / 1024;
  constexpr int XPW = (XPIECES + 3) / 4;
  constexpr int ZERO_OFF = 0;  // 512 zero bytes: a masked tap's fragment address lands here
  constexpr int X_OFF = 512;
  constexpr int HHI_OFF = X_OFF + 4 * XPW * 1024;
  constexpr int HLO_OFF = HHI_OFF + kVpHR * kVpPitch;
  constexpr int VEC_OFF = HLO_OFF + kVpHR * kVpPitch;  // b1, g1, be1, b2, g2, be2, lin_w
  constexpr int RED_OFF = VEC_OFF + 7 * kVpC * 4;       // row statistics [48 rows][4 waves]
  constexpr int IDX_OFF = RED_OFF + kVpHR * 4 * 4;      // bucket index per output row
  constexpr int SMEM = IDX_OFF + kVpBM * 4;
  static_assert(SMEM <= 163840, "LDS");
  static_assert(kVpPrefetchMax + XPW + 8 * kVpDepth <= 63, "vmcnt holds at most 63 outstanding loads");
  static_assert(kVpScratchOff == HHI_OFF && 4 * 1024 <= kVpHR * kVpPitch, "warm-up scratch slot");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (tile, predictor): with two predictors XCDs 0-3 run g = 0 and 4-7 g = 1 (round-robin dispatch;
  // speed only), so each XCD's L2 streams ONE predictor's 1.5 MB of weights
  int g = 0, tile = blockIdx.x;
  if (p.G == 2) {
    const int xcd = blockIdx.x & 7;
    g = xcd >> 2;
    tile = (blockIdx.x >> 3) * 4 + (xcd & 3);
  }
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  // ---- L2 warm-up: the workgroups of one XCD march through the same weight stream in lockstep, so
  // a ring load is one HBM round trip for the whole XCD (≈ 45–70 GB/s per CU measured). Each wave
  // first pulls a disjoint 1 KiB slice of its predictor's stream (1.5 MB, fits the XCD's 4 MB L2)
  // by LDS DMA into a scratch slot (HHI, unused until LN1): the XCD fetches the whole stream at once
  // and the rings then hit L2. Dispatch is round-robin over the XCDs (speed only, like g above).
  if (p.prefetch) {
    constexpr int kPieces = (int)(4 * kVpWaveBytes / 1024);
    const int xcd = blockIdx.x & 7, peers = ((int)gridDim.x - xcd + 7) / 8;
    const int me = (int)(blockIdx.x >> 3) * 4 + w, nw = peers * 4;
    const uint32_t gb = (uint32_t)g * 4u * kVpWaveBytes + (uint32_t)lane * 16u;
    for (int i = 0, pc = me; i < kVpPrefetchMax && pc < kPieces; ++i, pc += nw)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(smem + kVpScratchOff + w * 1024),
                                               16, gb + (uint32_t)pc * 1024u, 0, 0, 0);
  }
  if (tile >= p.ntiles) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS outlives the workgroup
    return;
  }
  const int M = p.M, L = p.L, m0 = tile * kVpBM;
  const int r16 = lane & 15, hi = lane >> 4;

  // ---- tap masks: bit t set when row + t - 1 lies in the row's own utterance
  auto taps = [&](int gm) {
    int v = 0;
    if (gm >= 0 && gm < M) {
      const int tpos = gm % L;
#pragma unroll
      for (int t = 0; t < 3; ++t) v |= ((unsigned)(tpos + t - 1) < (unsigned)L ? 1 : 0) << t;
    }
    return v;
  };
  int vm1[3], vm2[2];
#pragma unroll
  for (int nb = 0; nb < 3; ++nb) vm1[nb] = taps(m0 - 1 + nb * 16 + r16);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) vm2[nb] = taps(m0 + nb * 16 + r16);

  const float *vec = p.vec + (size_t)g * 7 * kVpC;
  for (int i = tid; i < 7 * kVpC / 4; i += 256)
    *reinterpret_cast<float4 *>(smem + VEC_OFF + 16 * i) = reinterpret_cast<const float4 *>(vec)[i];
  if (tid < 32) *reinterpret_cast<float4 *>(smem + ZERO_OFF + 16 * tid) = make_float4(0.f, 0.f, 0.f, 0.f);

  // ---- x tile (rows m0 - 2 .. m0 + 47) -> LDS by DMA, lane-linear pieces of 1 KiB
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const uint32_t xrow = (uint32_t)p.xs * 2u;
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int pc = w + 4 * i;
    const int o = pc * 1024 + lane * 16;
    const int r = o / kVpPitch, within = o - r * kVpPitch;
    const int gm = m0 - 2 + r;
    const bool ok = r < kVpXR && within < 512 && gm >= 0 && gm < M;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                             16, ok ? (uint32_t)gm * xrow + (uint32_t)within : kOOB, 0, 0, 0);
  }

  // ---- weight ring: k-step k (0..47: conv1 then conv2) = units 2k (w_hi), 2k + 1 (w_lo)
  const uint32_t wbase = (uint32_t)(g * 4 + w) * kVpWaveBytes;
  const uint32_t lane_off = (uint32_t)lane * 16u;
  bf16x8 pa[kVpDepth][2][4];
  auto load_at = [&](auto S, int k) {
    constexpr int s = decltype(S)::value;
    const uint32_t so = wbase + (uint32_t)(min(k, 2 * kVpKS - 1) * 2) * (uint32_t)kVpUnit;  // past the end: reload
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        pa[s][e][jb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                      wr, lane_off + (uint32_t)(jb * 1024), so + e * kVpUnit, 0));
    __builtin_amdgcn_sched_barrier(0);
  };
  vp_static_for<kVpDepth>([&](auto I) { load_at(I, decltype(I)::value); });

  auto bar = []() {
    __builtin_amdgcn_s_waitcnt(kVpLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * kVpDepth) : "memory");  // the x tile (older than the ring)
  bar();

  f32x4 acc1[4][3], acc2[4][2];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) acc1[jb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc2[jb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- conv1: B fragments from the x tile (row r16 + 16 nb + tap, channels 32 ks + 8 hi)
  auto bases1 = [&](int tap, int (&ad)[3]) {
    const int base = X_OFF + (r16 + tap) * kVpPitch + hi * 16;
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) ad[nb] = (base + nb * 16 * kVpPitch) & __builtin_amdgcn_sbfe(vm1[nb], tap, 1);
  };
  auto rd1 = [&](const int (&ad)[3], auto KSI, bf16x8 (&f)[3]) {
    constexpr int off = decltype(KSI)::value * 64;
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) f[nb] = *reinterpret_cast<const bf16x8 *>(smem + ad[nb] + off);
  };
  auto mma1 = [&](auto S, const bf16x8 (&f)[3]) {
    constexpr int s = decltype(S)::value;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int nb = 0; nb < 3; ++nb)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
          acc1[jb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[s][e][jb], f[nb], acc1[jb][nb], 0, 0, 0);
  };
  bf16x8 fa0[3], fa1[3];
  int bc[3], bn[3];
  bases1(0, bc);
  rd1(bc, std::integral_constant<int, 0>{}, fa0);
#pragma nounroll
  for (int tap = 0; tap < 3; ++tap) {
    bases1(tap + 1, bn);  // tap 3: every bit clear -> the zero slot (the read after the last k-step)
    vp_static_for<8>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value, s = ks % kVpDepth;
      if constexpr (ks + 1 < 8) {
        if constexpr (ks & 1)
          rd1(bc, std::integral_constant<int, ks + 1>{}, fa0);
        else
          rd1(bc, std::integral_constant<int, ks + 1>{}, fa1);
      } else {
        rd1(bn, std::integral_constant<int, 0>{}, fa0);
      }
      if constexpr (ks & 1)
        mma1(std::integral_constant<int, s>{}, fa1);
      else
        mma1(std::integral_constant<int, s>{}, fa0);
      load_at(std::integral_constant<int, s>{}, tap * 8 + ks + kVpDepth);
    });
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) bc[nb] = bn[nb];
  }

  // ---- row statistics over the 256 channels: a lane holds 16 of them (4 blocks x 4) for rows
  // r16 + 16 nb, the 4 lanes r16 + 16 hi of a wave 64, the 4 waves the rest (through LDS)
  float *red = reinterpret_cast<float *>(smem + RED_OFF);
  const float inv_n = 1.0f / (float)kVpC;
  auto row_reduce = [&](auto NBC, float *pv, float *tot) {
    constexpr int NB = decltype(NBC)::value;
    float t[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) t[nb] = __shfl_xor(pv[nb], 16, 64);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) pv[nb] += t[nb];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) t[nb] = __shfl_xor(pv[nb], 32, 64);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) red[(nb * 16 + r16) * 4 + w] = pv[nb] + t[nb];
    bar();
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const float4 r = *reinterpret_cast<const float4 *>(red + (nb * 16 + r16) * 4);
      tot[nb] = (r.x + r.y) + (r.z + r.w);
    }
    bar();  // red is reused by the next statistic
  };
  const float *V = reinterpret_cast<const float *>(smem + VEC_OFF);
  auto vec4 = [&](int which, int ch) { return *reinterpret_cast<const float4 *>(V + which * kVpC + ch); };

  // ---- LN1 -> h as bf16 hi / lo planes (fs2_vp_norm's arithmetic), rows 0..47 of the H tile
  {
    float part[3], mean[3], var[3];
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) {
      float sum = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const float4 b = vec4(0, w * 64 + jb * 16 + 4 * hi);
        f32x4 v = acc1[jb][nb];
        v[0] = fmaxf(v[0] + b.x, 0.f);
        v[1] = fmaxf(v[1] + b.y, 0.f);
        v[2] = fmaxf(v[2] + b.z, 0.f);
        v[3] = fmaxf(v[3] + b.w, 0.f);
        acc1[jb][nb] = v;
        sum += (v[0] + v[1]) + (v[2] + v[3]);
      }
      part[nb] = sum;
    }
    row_reduce(std::integral_constant<int, 3>{}, part, mean);
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) {
      mean[nb] *= inv_n;
      float ss = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        f32x4 d = acc1[jb][nb];
        d[0] -= mean[nb];
        d[1] -= mean[nb];
        d[2] -= mean[nb];
        d[3] -= mean[nb];
        acc1[jb][nb] = d;
        ss += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
      }
      part[nb] = ss;
    }
    row_reduce(std::integral_constant<int, 3>{}, part, var);
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) {
      const float rstd = 1.0f / sqrtf(var[nb] * inv_n + p.eps);
      const int row = nb * 16 + r16;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int ch = w * 64 + jb * 16 + 4 * hi;
        const float4 ga = vec4(1, ch), be = vec4(2, ch);
        const f32x4 d = acc1[jb][nb];
        const float h[4] = {d[0] * rstd * ga.x + be.x, d[1] * rstd * ga.y + be.y, d[2] * rstd * ga.z + be.z,
                            d[3] * rstd * ga.w + be.w};
        bf16x4 oh, ol;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          oh[q] = (bf16)h[q];
          ol[q] = (bf16)(h[q] - (float)oh[q]);
        }
        *reinterpret_cast<bf16x4 *>(smem + HHI_OFF + row * kVpPitch + ch * 2) = oh;
        *reinterpret_cast<bf16x4 *>(smem + HLO_OFF + row * kVpPitch + ch * 2) = ol;
      }
    }
  }
  bar();  // the H planes are visible

  // ---- conv2: output row j = r16 + 16 nb reads h rows j + tap (h row i <-> global m0 - 1 + i)
  auto bases2 = [&](int tap, int (&ah)[2], int (&al)[2]) {
    const int rel = (r16 + tap) * kVpPitch + hi * 16;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int keep = __builtin_amdgcn_sbfe(vm2[nb], tap, 1);
      ah[nb] = (HHI_OFF + rel + nb * 16 * kVpPitch) & keep;
      al[nb] = (HLO_OFF + rel + nb * 16 * kVpPitch) & keep;
    }
  };
  auto rd2 = [&](const int (&ah)[2], const int (&al)[2], auto KSI, bf16x8 (&fh)[2], bf16x8 (&fl)[2]) {
    constexpr int off = decltype(KSI)::value * 64;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      fh[nb] = *reinterpret_cast<const bf16x8 *>(smem + ah[nb] + off);
      fl[nb] = *reinterpret_cast<const bf16x8 *>(smem + al[nb] + off);
    }
  };
  auto mma2 = [&](auto S, const bf16x8 (&fh)[2], const bf16x8 (&fl)[2]) {
    constexpr int s = decltype(S)::value;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc2[jb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[s][0][jb], fh[nb], acc2[jb][nb], 0, 0, 0);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc2[jb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[s][1][jb], fh[nb], acc2[jb][nb], 0, 0, 0);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc2[jb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[s][0][jb], fl[nb], acc2[jb][nb], 0, 0, 0);
  };
  {
    bf16x8 fh0[2], fl0[2], fh1[2], fl1[2];
    int ahc[2], alc[2], ahn[2], aln[2];
    bases2(0, ahc, alc);
    rd2(ahc, alc, std::integral_constant<int, 0>{}, fh0, fl0);
#pragma nounroll
    for (int tap = 0; tap < 3; ++tap) {
      bases2(tap + 1, ahn, aln);
      vp_static_for<8>([&](auto KSI) {
        constexpr int ks = decltype(KSI)::value, s = ks % kVpDepth;
        if constexpr (ks + 1 < 8) {
          if constexpr (ks & 1)
            rd2(ahc, alc, std::integral_constant<int, ks + 1>{}, fh0, fl0);
          else
            rd2(ahc, alc, std::integral_constant<int, ks + 1>{}, fh1, fl1);
        } else {
          rd2(ahn, aln, std::integral_constant<int, 0>{}, fh0, fl0);
        }
        if constexpr (ks & 1)
          mma2(std::integral_constant<int, s>{}, fh1, fl1);
        else
          mma2(std::integral_constant<int, s>{}, fh0, fl0);
        load_at(std::integral_constant<int, s>{}, kVpKS + tap * 8 + ks + kVpDepth);
      });
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        ahc[nb] = ahn[nb];
        alc[nb] = aln[nb];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-the-end reloads

  // ---- LN2, Linear(256 -> 1), mask (fs2_vp_head's arithmetic)
  float dot[2];
  {
    float part[2], mean[2], var[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float sum = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const float4 b = vec4(3, w * 64 + jb * 16 + 4 * hi);
        f32x4 v = acc2[jb][nb];
        v[0] = fmaxf(v[0] + b.x, 0.f);
        v[1] = fmaxf(v[1] + b.y, 0.f);
        v[2] = fmaxf(v[2] + b.z, 0.f);
        v[3] = fmaxf(v[3] + b.w, 0.f);
        acc2[jb][nb] = v;
        sum += (v[0] + v[1]) + (v[2] + v[3]);
      }
      part[nb] = sum;
    }
    row_reduce(std::integral_constant<int, 2>{}, part, mean);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      mean[nb] *= inv_n;
      float ss = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        f32x4 d = acc2[jb][nb];
        d[0] -= mean[nb];
        d[1] -= mean[nb];
        d[2] -= mean[nb];
        d[3] -= mean[nb];
        acc2[jb][nb] = d;
        ss += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
      }
      part[nb] = ss;
    }
    row_reduce(std::integral_constant<int, 2>{}, part, var);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const float rstd = 1.0f / sqrtf(var[nb] * inv_n + p.eps);
      float sd = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int ch = w * 64 + jb * 16 + 4 * hi;
        const float4 ga = vec4(4, ch), be = vec4(5, ch), lw = vec4(6, ch);
        const f32x4 d = acc2[jb][nb];
        sd += (d[0] * rstd * ga.x + be.x) * lw.x + (d[1] * rstd * ga.y + be.y) * lw.y +
              (d[2] * rstd * ga.z + be.z) * lw.z + (d[3] * rstd * ga.w + be.w) * lw.w;
      }
      part[nb] = sd;
    }
    row_reduce(std::integral_constant<int, 2>{}, part, dot);
  }
  const bool embed = g == p.embed_g;
  int *idx = reinterpret_cast<int *>(smem + IDX_OFF);
  if (w == 0 && hi == 0) {
    const float lb = p.lin_b[g];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int j = nb * 16 + r16, gm = m0 + j;
      if (gm < M) {
        const int b = gm / L, t = gm - b * L;
        const float pv = (int64_t)t >= p.lens[b] ? 0.0f : dot[nb] + lb;
        if (!embed) {
          p.pred[(size_t)g * M + gm] = pv;
        } else {
          // fs2_variance_embed semantics: a target is bucketized as given (the prediction kept);
          // otherwise the prediction is scaled by control first
          const float val = p.target != nullptr ? p.target[gm] : pv * p.control;
          p.pred[(size_t)g * M + gm] = p.target != nullptr ? pv : val;
          int lo = 0, hb = p.nb;  // torch.bucketize(val, bins, right=False)
          while (lo < hb) {
            const int mid = (lo + hb) >> 1;
            if (p.bins[mid] < val) lo = mid + 1; else hb = mid;
          }
          idx[j] = lo;
        }
      }
    }
  }
  if (!embed) return;
  bar();
  // x_out = x + table[idx] over the tile's rows: x from the LDS tile (row j + 2), 16 bytes a lane
  char *ob = reinterpret_cast<char *>(p.xo);
  const uint32_t orow = (uint32_t)p.xos * 2u;
#pragma unroll
  for (int i = tid; i < kVpBM * 32; i += 256) {
    const int j = i >> 5, ch = i & 31;
    if (m0 + j < M) {
      float a[8], e[8];
      load8(reinterpret_cast<const bf16 *>(smem + X_OFF + (j + 2) * kVpPitch + ch * 16), a);
      load8(p.table + (size_t)idx[j] * kVpC + ch * 8, e);
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] += e[q];
      store8(reinterpret_cast<bf16 *>(ob + (size_t)(m0 + j) * orow + ch * 16), a);
    }
  }
}

}  // namespace

extern "C" int64_t fs2_vp_fused_weight_elems(int G) { return (int64_t)G * 4 * kVpWaveBytes / 2; }

extern "C" int fs2_vp_fused(const fs2_vp_fused_desc *d, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->vec == nullptr || d->lin_b == nullptr ||
      d->lens == nullptr || d->pred == nullptr)
    return FS2_EINVAL;
  if (d->B < 0 || d->L <= 0 || d->x_row_stride < kVpC || (d->x_row_stride & 7)) return FS2_EINVAL;
  if (!(d->G == 1 || d->G == 2) || d->embed_group < -1 || d->embed_group >= d->G) return FS2_EINVAL;
  if (d->embed_group >= 0) {
    if (d->x_out == nullptr || d->x_out == d->x || d->bins == nullptr || d->table == nullptr || d->n_bins < 2 ||
        d->x_out_row_stride < kVpC || (d->x_out_row_stride & 7))
      return FS2_EINVAL;
  }
  const int64_t M64 = (int64_t)d->B * d->L;
  if (M64 == 0) return FS2_OK;
  if (M64 * d->x_row_stride * 2 >= (1LL << 31)) return FS2_EUNSUPPORTED;
  VpArgs p{};
  p.x = reinterpret_cast<const bf16 *>(d->x);
  p.xs = d->x_row_stride;
  p.x_bytes = (uint32_t)(M64 * d->x_row_stride * 2);
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.w_bytes = (uint32_t)(fs2_vp_fused_weight_elems(d->G) * 2);
  p.vec = d->vec;
  p.lin_b = d->lin_b;
  p.eps = d->ln_eps;
  p.M = (int)M64;
  p.L = d->L;
  p.G = d->G;
  p.ntiles = (int)((M64 + kVpBM - 1) / kVpBM);
  p.lens = d->lens;
  p.pred = d->pred;
  p.embed_g = d->embed_group;
  p.xo = reinterpret_cast<bf16 *>(d->x_out);
  p.xos = d->x_out_row_stride;
  p.target = d->target;
  p.control = d->control;
  p.bins = d->bins;
  p.nb = d->n_bins - 1;
  p.table = d->table;
  static const int prefetch = [] {
    const char *e = getenv("FS2_VP_PREFETCH");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  p.prefetch = prefetch;
  const int nwg = d->G == 2 ? 8 * ((p.ntiles + 3) / 4) : p.ntiles;
  hipLaunchKernelGGL(vp_fused_kernel, dim3(nwg), dim3(256), 0, as_stream(stream), p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_vp_norm(const float *y, int64_t y_row_stride, int M, int G, int C, const float *gamma,
                           const float *beta, float eps, void *out, int64_t out_row_stride, fs2_stream_t stream) {
  if (y == nullptr || gamma == nullptr || beta == nullptr || out == nullptr) return FS2_EINVAL;
  if (M < 0 || G <= 0) return FS2_EINVAL;
  if (C != kC) return FS2_EUNSUPPORTED;
  if (y_row_stride < (int64_t)G * C || (y_row_stride & 3) || out_row_stride < (int64_t)G * 2 * C || (out_row_stride & 7))
    return FS2_EINVAL;
  if (M == 0) return FS2_OK;
  const int64_t items = (int64_t)M * G;
  hipLaunchKernelGGL(vp_norm_kernel, dim3((unsigned)((items + 7) / 8)), dim3(256), 0, as_stream(stream), y,
                     y_row_stride, M, G, gamma, beta, eps, reinterpret_cast<bf16 *>(out), out_row_stride);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_vp_head(const float *y, int64_t y_row_stride, int B, int T, int G, int C, const float *gamma,
                           const float *beta, float eps, const float *lin_w, const float *lin_b, const int64_t *lens,
                           float *pred, int embed_group, void *x, int x_dtype, int64_t x_row_stride, int D,
                           const float *target, float control, const float *bins, int n_bins, const float *table,
                           fs2_stream_t stream) {
  if (y == nullptr || gamma == nullptr || beta == nullptr || lin_w == nullptr || lin_b == nullptr ||
      lens == nullptr || pred == nullptr)
    return FS2_EINVAL;
  if (B < 0 || T < 0 || G <= 0 || embed_group >= G) return FS2_EINVAL;
  if (C != kC) return FS2_EUNSUPPORTED;
  if (y_row_stride < (int64_t)G * C || (y_row_stride & 3)) return FS2_EINVAL;
  if (embed_group >= 0) {
    if (x == nullptr || bins == nullptr || table == nullptr || n_bins < 2 || D <= 0 || (D & 7) ||
        x_row_stride < D || (x_row_stride & 7))
      return FS2_EINVAL;
    if (x_dtype != FS2_F32 && x_dtype != FS2_BF16) return FS2_EUNSUPPORTED;
  }
  const int64_t M64 = (int64_t)B * T;
  if (M64 > 0x7fffffffLL) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;
  const int M = (int)M64;
  const dim3 grid((unsigned)(((int64_t)M * G + 7) / 8));
  hipStream_t s = as_stream(stream);
  if (embed_group >= 0 && x_dtype == FS2_F32)
    hipLaunchKernelGGL(vp_head_kernel<float>, grid, dim3(256), 0, s, y, y_row_stride, T, M, G, gamma, beta, eps, lin_w,
                       lin_b, lens, pred, embed_group, reinterpret_cast<float *>(x), x_row_stride, D, target, control,
                       bins, n_bins - 1, table);
  else
    hipLaunchKernelGGL(vp_head_kernel<bf16>, grid, dim3(256), 0, s, y, y_row_stride, T, M, G, gamma, beta, eps, lin_w,
                       lin_b, lens, pred, embed_group, reinterpret_cast<bf16 *>(x), x_row_stride, D, target, control,
                       bins, n_bins - 1, table);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
