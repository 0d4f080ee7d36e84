// Weight-streamed Conv1d (gfx950 / CDNA4) for the PostNet's 512 -> 512, k = 5 convolutions
// (transformer/Layers.py:92-137: Conv1d + BatchNorm (folded on the host) + tanh):
//
//   y[m, n] = tanh( sum_{tap, c} x[m + tap - pad, c] * w[n, c, tap] + b[n] )   per-sequence zero taps
//
// The structure of the fused FFN's GEMM1 (ffn.hip), for N = 512: a workgroup owns 112 rows and all
// 512 output columns; 8 waves, two per SIMD, wave w owns output columns 64w .. 64w+63 (MFMA A side,
// 4 row blocks) x the 112 rows (B side, 7 blocks), its 16x16 f32 accumulators in AGPRs.
//
// * Weights never touch LDS: each wave streams its own 64 rows from the fragment-ordered buffer
//   (ops.pack_wconv_weight: a "unit" = 64 rows x 32 channels = 4 KiB contiguous; one coalesced
//   16-byte-per-lane load per 1 KiB row block) straight into A-operand registers, 4 units ahead
//   (the other wave on the SIMD hides the rest of the latency).
// * The x tile (112 + KS - 1 rows x 512 channels) is DMA'd to LDS once at a 1056-byte row pitch
//   (1024 + 32): a B fragment's 16 rows fall in 16 distinct bank groups for any tap shift, so a
//   unit's k-step is the ds_read immediate. Rows whose tap leaves the sequence (padded [B, T]
//   rows: t mod T) read a 1 KiB zero region at LDS 0 (per-lane tap-validity bits, address & mask).
// * Epilogue: + bias, tanh, bf16; staged through LDS (pitch 1040: the 8-byte column writes 2-way)
//   and stored as whole 1 KiB rows.
#include <type_traits>
#include <utility>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

constexpr int kUnitB = 4096;  // bytes of one wave unit: 4 row blocks x 64 lanes x 16 B

struct WconvArgs {
  const bf16 *x;
  int64_t xs;       // x row stride (elements)
  const bf16 *w;    // fragment order [N/64][KS][Cin/32][4][64][8]
  const float *bias;
  bf16 *out;
  int64_t os;
  int B, T, M, pad;
  uint32_t x_bytes, w_bytes;
};

template <int N, typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

constexpr int kLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0) the compiler's wait-count pass sees

// CIN % 32 != 0 (the PostNet's first conv, 80 -> 512): the K dimension is (tap, channel) flattened,
// k = tap * CIN + c, in 32-wide steps ("flat" units); a lane group's 8 consecutive k stay inside one
// tap (CIN % 8 == 0), so each lane addresses its own (row + tap, channel) per unit.
template <int KS, int CIN, int WQ>
__global__ __launch_bounds__(512 / WQ, 1) void wconv_kernel(WconvArgs p) {
  constexpr bool FLAT = CIN % 32 != 0;
  static_assert(CIN % 8 == 0, "8-channel lane groups");
  // WQ: 64-column quads per wave (1: 8 waves, two per SIMD; 2: 4 waves, 128 columns each)
  constexpr int MB = 7, BM = 16 * MB, NWV = 8 / WQ, NT = 64 * NWV, NCOL = 512, JB = 4 * WQ;
  constexpr int XROWS = BM + KS - 1;
  constexpr int XPITCH = FLAT ? CIN * 2 + 16 : CIN * 2 + 32;  // 80 ch: 176 B, rows in distinct bank quads
  constexpr int XPIECES = (XROWS * XPITCH + 1023) / 1024;
  constexpr int XP_PER_WAVE = (XPIECES + NWV - 1) / NWV;
  constexpr int NKS = FLAT ? 1 : CIN / 32;             // k-steps (units) per tap
  constexpr int ZBYTES = FLAT ? 64 : NKS * 64;          // zero region: a masked row reads base 0 + 64 ks
  constexpr int X_OFF = ZBYTES;
  constexpr int OPITCH = NCOL * 2 + 16;                 // output staging pitch
  // the x region doubles as the output staging area (sized for the larger of the two)
  constexpr int XREG = NWV * XP_PER_WAVE * 1024 > BM * OPITCH ? NWV * XP_PER_WAVE * 1024 : BM * OPITCH;
  constexpr int BIAS_OFF = X_OFF + XREG;
  constexpr int SMEM = BIAS_OFF + NCOL * 4;
  static_assert(SMEM <= 163840, "LDS");
  constexpr int DEPTH = WQ == 1 ? 4 : 2;
  static_assert(FLAT || NKS % DEPTH == 0, "static ring slots");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = p.M, T = p.T, pad = p.pad;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int hrow0 = lane & 15, hi = lane >> 4;

  // tap validity (padded rows: position t mod T in a sequence of T frames)
  int vmask[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + mb * 16 + hrow0;
    const int tpos = m < M ? m % T : 0, tlen = m < M ? T : 0;
    int v = 0;
#pragma unroll
    for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(tpos + tap - pad) < (unsigned)tlen ? 1 : 0) << tap;
    vmask[mb] = v;
  }
  for (int i = tid; i < ZBYTES / 16; i += NT)
    *reinterpret_cast<float4 *>(smem + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < NCOL / 4)
    *reinterpret_cast<float4 *>(smem + BIAS_OFF + 16 * tid) = reinterpret_cast<const float4 *>(p.bias)[tid];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) asm volatile("" ::"v"(vmask[mb]));

  // x tile -> LDS once (lane-linear 1 KiB pieces at the padded pitch)
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t xrow = (uint32_t)p.xs * 2u;
#pragma unroll
  for (int i = 0; i < XP_PER_WAVE; ++i) {
    const int pc = w + NWV * i;
    const int o = pc * 1024 + lane * 16;
    const int r = o / XPITCH, within = o - r * XPITCH;
    const int gm = m0 - pad + r;
    const bool ok = r < XROWS && within < CIN * 2 && gm >= 0 && gm < M;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                             16, ok ? (uint32_t)gm * xrow + (uint32_t)within : kOOB, 0, 0, 0);
  }

  // weight stream: unit u = tap * NKS + ks of this wave's 64 rows; past the last unit a harmless reload
  constexpr int NU = FLAT ? (KS * CIN + 31) / 32 : KS * NKS;
  const uint32_t wbase = (uint32_t)(w * WQ * NU) * (uint32_t)kUnitB, lane_off = (uint32_t)lane * 16u;
  bf16x8 pa[DEPTH][JB];
  auto load_at = [&](auto S, int u) {
    constexpr int s = decltype(S)::value;
    const uint32_t so = wbase + (uint32_t)(u < NU ? u : 0) * (uint32_t)kUnitB;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) {  // quad jb / 4 of the wave: NU units further in the buffer
      auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, lane_off + (jb & 3) * 1024,
                                                     so + (uint32_t)((jb >> 2) * NU) * (uint32_t)kUnitB, 0);
      pa[s][jb] = __builtin_bit_cast(bf16x8, v);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  static_for<DEPTH>([&](auto S) { load_at(S, decltype(S)::value); });

  auto bases_x = [&](int tap, int (&ad)[MB]) {
    const int base = X_OFF + (hrow0 + tap) * XPITCH + hi * 16;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) ad[mb] = (base + mb * 16 * XPITCH) & __builtin_amdgcn_sbfe(vmask[mb], tap, 1);
  };
  bf16x8 f0[MB], f1[MB];
  auto issue_x = [&](const int (&ad)[MB], auto KSI, bf16x8 (&f)[MB]) {
    constexpr int off = decltype(KSI)::value * 64;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) f[mb] = *reinterpret_cast<const bf16x8 *>(smem + ad[mb] + off);
  };
  f32x4 acc[JB][MB];
#pragma unroll
  for (int i = 0; i < JB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&fa)[JB], const bf16x8 (&fb)[MB]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int jb = 0; jb < JB; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[jb], fb[mb], acc[jb][mb], 0, 0, 0);
  };

  // x tile landed (the ring's loads may stay in flight), zero region and bias stored; visible
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * DEPTH) : "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();
  if constexpr (FLAT) {
    // unit u, lane group hi: k = 32u + 8hi -> (tap, channel); k >= KS * CIN: zero weights, any
    // in-tile address (the zero region)
    auto bases_flat = [&](int u, int (&ad)[MB]) {
      const int k = 32 * u + 8 * hi;
      const int tap = k / CIN, c = k - tap * CIN;
      const int base = X_OFF + (hrow0 + tap) * XPITCH + c * 2;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        ad[mb] = tap < KS ? (base + mb * 16 * XPITCH) & __builtin_amdgcn_sbfe(vmask[mb], tap, 1) : 0;
    };
    int ad[MB];
    bases_flat(0, ad);
    issue_x(ad, std::integral_constant<int, 0>{}, f0);
    static_for<NU>([&](auto UI) {
      constexpr int u = decltype(UI)::value;
      if constexpr (u + 1 < NU) {
        bases_flat(u + 1, ad);
        if constexpr (u & 1)
          issue_x(ad, std::integral_constant<int, 0>{}, f0);
        else
          issue_x(ad, std::integral_constant<int, 0>{}, f1);
      }
      if constexpr (u & 1)
        mma(pa[u % DEPTH], f1);
      else
        mma(pa[u % DEPTH], f0);
      load_at(std::integral_constant<int, u % DEPTH>{}, u + DEPTH);
    });
  } else {
  int bxc[MB], bxn[MB];
  bases_x(0, bxc);
  issue_x(bxc, std::integral_constant<int, 0>{}, f0);
#pragma nounroll
  for (int tap = 0; tap < KS; ++tap) {
    bases_x(tap + 1, bxn);  // tap KS: every row masked (zero region), a harmless read
    static_for<NKS>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value;
      if constexpr (ks + 1 < NKS) {
        if constexpr (ks & 1)
          issue_x(bxc, std::integral_constant<int, ks + 1>{}, f0);
        else
          issue_x(bxc, std::integral_constant<int, ks + 1>{}, f1);
      } else {
        issue_x(bxn, std::integral_constant<int, 0>{}, f0);
      }
      if constexpr (ks & 1)
        mma(pa[ks % DEPTH], f1);
      else
        mma(pa[ks % DEPTH], f0);
      load_at(std::integral_constant<int, ks % DEPTH>{}, tap * NKS + ks + DEPTH);
    });
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) bxc[mb] = bxn[mb];
  }
  }

  // epilogue: + bias, tanh, bf16 -> LDS staging (the x region) -> whole-row stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();
#pragma unroll
  for (int nb = 0; nb < JB; ++nb) {
    const int n = w * 64 * WQ + nb * 16 + 4 * hi;
    const float4 bb = *reinterpret_cast<const float4 *>(smem + BIAS_OFF + 4 * n);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[nb][mb];
      bf16x4 o;
      o[0] = (bf16)tanhf(v[0] + bb.x);
      o[1] = (bf16)tanhf(v[1] + bb.y);
      o[2] = (bf16)tanhf(v[2] + bb.z);
      o[3] = (bf16)tanhf(v[3] + bb.w);
      *reinterpret_cast<bf16x4 *>(smem + X_OFF + (hrow0 + mb * 16) * OPITCH + n * 2) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = NCOL * 2 / 16;  // 16-byte chunks per output row
  char *ob = reinterpret_cast<char *>(p.out);
  const uint32_t orow = (uint32_t)p.os * 2u;
#pragma unroll 2
  for (int i = tid; i < BM * CPR; i += NT) {
    const int m = i / CPR, ch = i - m * CPR;
    if (m0 + m < M)
      *reinterpret_cast<uint4 *>(ob + (size_t)(m0 + m) * orow + ch * 16) =
          *reinterpret_cast<const uint4 *>(smem + X_OFF + m * OPITCH + ch * 16);
  }
}

}  // namespace

extern "C" int64_t fs2_wconv_weight_elems(int KS, int Cin, int N) { return (int64_t)N * ((KS * Cin + 31) / 32 * 32); }

extern "C" int fs2_wconv(const fs2_wconv_desc *d, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->bias == nullptr || d->out == nullptr)
    return FS2_EINVAL;
  if (d->B < 0 || d->T < 0 || d->pad < 0 || d->x_row_stride < d->Cin || (d->x_row_stride & 7) ||
      d->out_row_stride < d->N || (d->out_row_stride & 7))
    return FS2_EINVAL;
  if (!(d->Cin == 512 || d->Cin == 80) || d->N != 512 || d->KS != 5 || d->pad > d->KS - 1 ||
      d->epilogue != FS2_EPI_BIAS_TANH)
    return FS2_EUNSUPPORTED;
  if (d->x == d->out) return FS2_EINVAL;  // other tiles re-read x rows (halo)
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 == 0) return FS2_OK;
  const int64_t xb = M64 * d->x_row_stride * 2;
  if (xb >= (1LL << 31) || M64 > 0x7fffff00LL) return FS2_EUNSUPPORTED;
  WconvArgs p;
  p.x = reinterpret_cast<const bf16 *>(d->x);
  p.xs = d->x_row_stride;
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.bias = d->bias;
  p.out = reinterpret_cast<bf16 *>(d->out);
  p.os = d->out_row_stride;
  p.B = d->B;
  p.T = d->T;
  p.M = (int)M64;
  p.pad = d->pad;
  p.x_bytes = (uint32_t)xb;
  p.w_bytes = (uint32_t)(fs2_wconv_weight_elems(d->KS, d->Cin, d->N) * 2);
  const int nwg = (int)((M64 + 111) / 112);
#ifndef WCONV_WQ
#define WCONV_WQ 1  // 8 waves x 64 columns (2 quads per wave: 224 accumulators + the ring spill; analysis only)
#endif
  if (d->Cin == 80)
    hipLaunchKernelGGL((wconv_kernel<5, 80, 1>), dim3(nwg), dim3(512), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((wconv_kernel<5, 512, WCONV_WQ>), dim3(nwg), dim3(512 / WCONV_WQ), 0, as_stream(stream), p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
