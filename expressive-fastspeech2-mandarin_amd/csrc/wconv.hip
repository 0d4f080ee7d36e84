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
  const int2 *row_pos;     // packed rows: {frame, length} per row (NULL: padded [B, T] rows)
  const int32_t *rows_dev; // packed rows: the active row count (device)
  int out_sc1;             // write-through output rows (conv_common.h store16_out)
  // TAIL (the PostNet's last two convs in one launch): the 512 -> 80 conv + residual on this
  // conv's output tile; w2 in pn_tail's k-step-major order, f32 out2 = conv + bias2 + res
  const bf16 *w2;
  const float *bias2;
  const float *res;
  int64_t rs;
  float *out2;
  int64_t os2;
  uint32_t w2_bytes;
};

// position and length of row m's sequence: packed rows from row_pos, padded rows t = m mod T
__device__ __forceinline__ void seq_pos(const int2 *row_pos, int m, int T, int &tpos, int &tlen) {
  if (row_pos != nullptr) {
    const int2 q = row_pos[m];
    tpos = q.x;
    tlen = q.y;
  } else {
    tpos = m % T;
    tlen = T;
  }
}

template <int N, typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

constexpr int kLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0) the compiler's wait-count pass sees

// tanh for the bf16 epilogues: 1 - 2 / (1 + e^(2x)) with the hardware exp2 / reciprocal (5
// instructions; libm tanhf is ~35 with its range branches, and the PostNet epilogues evaluate
// 57k of them per workgroup). |error| <= ~2e-7 absolute: far below the bf16 rounding of the result;
// saturates to +-1 (e^(2x) = inf -> 1, 0 -> -1).
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2 log2(e)
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
}

// The fused PostNet tail (wconv_kernel<5, 512, 1, true>): this conv's 112 output rows (y, + bias,
// tanh) go to LDS at the x-tile pitch and feed the 512 -> 80 conv + residual (transformer/Layers.py
// :129-137, fastspeech2.py:136) on the workgroup's TB = 108 middle rows -- pn_tail_kernel's k-step
// order (so the result is bit-identical to the two launches) without the 28 MB y round trip or
// its launch. LDS bandwidth bounds this part (every wave reads the k-step's 5 KiB of weight
// fragments), so 4 waves, one per SIMD, own 2 row blocks x the 5 column blocks each (27 KiB of
// fragment reads per k-step instead of 42 with one row block per wave); the other 4 waves DMA
// the weight ring (2 k-steps x 5 KiB per stage, 3 stages).
#ifndef WCONV_TAIL_ABLATE
#define WCONV_TAIL_ABLATE 0  // analysis builds only: 1 skips the tail MFMA loop, 2 the whole tail (timing)
#endif
template <int X_OFF, int XPITCH, int BIAS_OFF, int W_OFF, int B_OFF>
__device__ __forceinline__ void tail_epilogue(const WconvArgs &p, const f32x4 (&acc)[4][7], char *smem, int m0, int M,
                                              int T, int w, int lane) {
  constexpr int MB = 7, KS = 5, NB = 5, KPS = 2, NST = 3, STG = KPS * NB * 1024, NKS = 16, NS = KS * NKS / KPS;
  constexpr int TB = 16 * MB - (KS - 1);
  const int hrow0 = lane & 15, hi = lane >> 4;
  if (WCONV_TAIL_ABLATE & 2) return;
  const rsrc_t w2r = make_rsrc(p.w2, p.w2_bytes);
  // waves 4..7 DMA a stage's 10 pieces: 3, 3, 2, 2
  const int dw = w - 4, npc = dw < 2 ? 3 : 2;
  auto wdma = [&](int st_idx) {
    if (dw >= 0) {
      char *st = smem + W_OFF + (st_idx % NST) * STG;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int pc = dw + 4 * j;
        if (j < npc)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(w2r, (__attribute__((address_space(3))) void *)(st + pc * 1024), 16,
                                                   (uint32_t)(st_idx * KPS * NB + pc) * 1024u + (uint32_t)lane * 16u, 0,
                                                   0, 0);
      }
    }
  };
  auto wait_stages = [&](bool one_in_flight) {  // this wave's pieces of the older stages landed
    if (!one_in_flight)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (npc == 3)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  };
  wdma(0);
  wdma(1);
  if (w == 3 && lane < 20)
    *reinterpret_cast<float4 *>(smem + B_OFF + 16 * lane) = reinterpret_cast<const float4 *>(p.bias2)[lane];
  // y = bf16(tanh(acc + b)) at the x pitch: row r of the tile is row m0 + r
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = w * 64 + nb * 16 + 4 * hi;
    const float4 bb = *reinterpret_cast<const float4 *>(smem + BIAS_OFF + 4 * n);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[nb][mb];
      bf16x4 o;
      o[0] = (bf16)tanh_fast(v[0] + bb.x);
      o[1] = (bf16)tanh_fast(v[1] + bb.y);
      o[2] = (bf16)tanh_fast(v[2] + bb.z);
      o[3] = (bf16)tanh_fast(v[3] + bb.w);
      *reinterpret_cast<bf16x4 *>(smem + X_OFF + (hrow0 + mb * 16) * XPITCH + n * 2) = o;
    }
  }
  // waves 0..3: tail rows i = 32 w + 16 j + hrow0 (j = 0, 1; i < TB), row g = m0 + 2 + i; tap t
  // reads tile row i + t
  int vt[2] = {0, 0}, ri[2], gi[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ri[j] = 32 * w + 16 * j + hrow0;
    gi[j] = m0 + (KS - 1) / 2 + ri[j];
    if (w < 4 && ri[j] < TB && gi[j] < M) {
      int tpos, tlen;
      seq_pos(p.row_pos, gi[j], T, tpos, tlen);
#pragma unroll
      for (int tap = 0; tap < KS; ++tap) vt[j] |= ((unsigned)(tpos + tap - 2) < (unsigned)tlen ? 1 : 0) << tap;
    }
  }
  f32x4 at[NB][2];
#pragma unroll
  for (int b = 0; b < NB; ++b) at[b][0] = at[b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // software-pipelined: stage st + 1's fragments are read (after its barrier) before stage st's
  // 20 MFMAs issue, so the LDS latency hides under them; the ring is 3 stages deep (DMA two ahead)
  struct Frags {
    bf16x8 fa[KPS][NB], fb[KPS][2];
  };
  auto read_stage = [&](int st, Frags &f) {
    const char *sp = smem + W_OFF + (st % NST) * STG;
#pragma unroll
    for (int q = 0; q < KPS; ++q) {
      const int u = st * KPS + q, tap = u >> 4, ks = u & 15;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ad = (X_OFF + (ri[j] + tap) * XPITCH + hi * 16) & __builtin_amdgcn_sbfe(vt[j], tap, 1);
        f.fb[q][j] = *reinterpret_cast<const bf16x8 *>(smem + ad + ks * 64);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) f.fa[q][b] = *reinterpret_cast<const bf16x8 *>(sp + (q * NB + b) * 1024 + lane * 16);
    }
  };
  auto mma_stage = [&](const Frags &f) {
#pragma unroll
    for (int q = 0; q < KPS; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int b = 0; b < NB; ++b) at[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.fa[q][b], f.fb[q][j], at[b][j], 0, 0, 0);
  };
  wdma(2);
  asm volatile("" ::: "memory");
  // stage 0 landed (stages 1 and 2 may stay in flight)
  if (npc == 3)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();  // y rows, tail bias, stage 0 visible
  Frags F0, F1;
  if (w < 4) read_stage(0, F0);
  auto step = [&](int st, Frags &cur, Frags &nxt) {
    if (st + 1 < NS) {
      wait_stages(st + 2 < NS);  // stage st + 1 landed (st + 2 may stay in flight)
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // ... visible; every wave's reads of stage st's slot are done
      __builtin_amdgcn_sched_barrier(0);
      if (st + NST < NS) wdma(st + NST);  // into stage st's slot
      if (w < 4) read_stage(st + 1, nxt);
    }
    if (w < 4) mma_stage(cur);
  };
#pragma nounroll
  for (int st = 0; st < NS; st += 2) {
    step(st, F0, F1);
    step(st + 1, F1, F0);
  }
  // + bias2 + residual, f32 rows (lane: row g, columns 16 b + 4 hi .. + 3)
  if (w < 4) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (ri[j] < TB && gi[j] < M) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int n = b * 16 + 4 * hi;
          const float4 bb = *reinterpret_cast<const float4 *>(smem + B_OFF + 4 * n);
          const float4 r = *reinterpret_cast<const float4 *>(p.res + (size_t)gi[j] * p.rs + n);
          const f32x4 v = at[b][j];
          *reinterpret_cast<float4 *>(p.out2 + (size_t)gi[j] * p.os2 + n) =
              make_float4((v[0] + bb.x) + r.x, (v[1] + bb.y) + r.y, (v[2] + bb.z) + r.z, (v[3] + bb.w) + r.w);
        }
      }
    }
  }
}

// CIN % 32 != 0 (the PostNet's first conv, 80 -> 512): the K dimension is (tap, channel) flattened,
// k = tap * CIN + c, in 32-wide steps ("flat" units); a lane group's 8 consecutive k stay inside one
// tap (CIN % 8 == 0), so each lane addresses its own (row + tap, channel) per unit.
template <int KS, int CIN, int WQ, bool TAIL = false>
__global__ __launch_bounds__(512 / WQ, 1) void wconv_kernel(WconvArgs p) {
  constexpr bool FLAT = CIN % 32 != 0;
  static_assert(!TAIL || (KS == 5 && CIN == 512 && WQ == 1), "the fused tail: the PostNet's 512 -> 512 -> 80");
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
  // TAIL: the 512 -> 80 conv's weight ring (NST stages of 2 k-steps x 5 fragment blocks) + bias
  constexpr int T_NB = 5, T_KPS = 2, T_NST = 3, T_STG = T_KPS * T_NB * 1024;
  constexpr int T_W_OFF = BIAS_OFF + NCOL * 4;
  constexpr int T_B_OFF = T_W_OFF + T_NST * T_STG;
  constexpr int SMEM = TAIL ? T_B_OFF + 80 * 4 : BIAS_OFF + NCOL * 4;
  static_assert(SMEM <= 163840, "LDS");
  constexpr int DEPTH = WQ == 1 ? 4 : 2;
  static_assert(FLAT || NKS % DEPTH == 0, "static ring slots");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M, T = p.T, pad = p.pad;
  // TAIL: a workgroup's 112 rows of this conv's output feed TB = 108 rows of the tail conv (its
  // taps reach 2 rows either side), so workgroups step by 108 and start 2 rows early
  constexpr int TB = TAIL ? BM - (KS - 1) : BM;
  if ((int)blockIdx.x * TB >= M) return;
  const int m0 = (int)blockIdx.x * TB - (TAIL ? (KS - 1) / 2 : 0);
  const int hrow0 = lane & 15, hi = lane >> 4;

  // tap validity (padded rows: position t mod T in a sequence of T frames; packed: row_pos)
  int vmask[MB];
  int2 rq[MB];  // packed rows: every block's row_pos entry loaded before any is used (one wait)
  if (p.row_pos != nullptr) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) rq[mb] = p.row_pos[min(max(m0 + mb * 16 + hrow0, 0), M - 1)];
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + mb * 16 + hrow0;
    int tpos = 0, tlen = 0;
    if (m >= 0 && m < M) {
      if (p.row_pos != nullptr) {
        tpos = rq[mb].x;
        tlen = rq[mb].y;
      } else {
        tpos = m % T;
        tlen = T;
      }
    }
    int v = 0;
#pragma unroll
    for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(tpos + tap - pad) < (unsigned)tlen ? 1 : 0) << tap;
    vmask[mb] = v;
  }
  for (int i = tid; i < ZBYTES / 16; i += NT)
    *reinterpret_cast<float4 *>(smem + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  // bias -> LDS by LDS-DMA (1 KiB pieces, waves 0..1): no load-to-store wait before the x tile DMA
  if (w < NCOL / 256)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(p.bias, NCOL * 4),
                                             (__attribute__((address_space(3))) void *)(smem + BIAS_OFF + w * 1024), 16,
                                             (uint32_t)(w * 1024 + lane * 16), 0, 0, 0);
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
  if constexpr (TAIL) {
    tail_epilogue<X_OFF, XPITCH, BIAS_OFF, T_W_OFF, T_B_OFF>(p, acc, smem, m0, M, T, w, lane);
    return;
  } else {
#pragma unroll
  for (int nb = 0; nb < JB; ++nb) {
    const int n = w * 64 * WQ + nb * 16 + 4 * hi;
    const float4 bb = *reinterpret_cast<const float4 *>(smem + BIAS_OFF + 4 * n);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[nb][mb];
      bf16x4 o;
      o[0] = (bf16)tanh_fast(v[0] + bb.x);
      o[1] = (bf16)tanh_fast(v[1] + bb.y);
      o[2] = (bf16)tanh_fast(v[2] + bb.z);
      o[3] = (bf16)tanh_fast(v[3] + bb.w);
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
      store16_out(ob, (uint32_t)(m0 + m) * orow + (uint32_t)ch * 16u,
                  *reinterpret_cast<const uint4 *>(smem + X_OFF + m * OPITCH + ch * 16), p.out_sc1);
  }
  }
}


// The PostNet's first two convolutions in ONE launch (transformer/Layers.py:92-137, layers 0 and 1):
//   y1 = tanh(conv_k5(mel; w1) + b1)   80 -> 512      (K = (tap, channel) flattened: 13 units)
//   y2 = tanh(conv_k5(y1; w2) + b2)    512 -> 512
// A workgroup owns BM = 112 rows of y2; it computes y1 on the 116 rows its taps read (m0-2 ..
// m0+113; the 4 halo rows recomputed, 3.6 %) from a 120-row mel tile, keeps y1 in LDS as the
// second conv's x tile (bf16, the wconv pitch) and runs wconv's main loop on it. The 28 MB y1
// write + re-read and the second launch's x-tile prologue (116 KB per workgroup from HBM) are gone.
struct PnHeadArgs {
  const bf16 *x;  // mel (bf16) [M, >= 80]
  int64_t xs;
  const bf16 *w1, *w2;
  const float *b1, *b2;
  bf16 *out;
  int64_t os;
  int T, M, pad;
  uint32_t x_bytes, w1_bytes, w2_bytes;
  const int2 *row_pos;
  const int32_t *rows_dev;
  int out_sc1;
};

__global__ __launch_bounds__(512, 1) void pn_head_kernel(PnHeadArgs p) {
  constexpr int KS = 5, CIN1 = 80, NCOL = 512, MB = 7, BM = 112, NWV = 8, NT = 512, JB = 4, DEPTH = 4;
  constexpr int YR = BM + KS - 1;            // y1 rows: m0 - 2 .. m0 + 113
  constexpr int XR = BM + 2 * (KS - 1);      // mel rows: m0 - 4 .. m0 + 115
  constexpr int YPITCH = NCOL * 2 + 32;      // 1056: conflict-free fragment reads for any tap
  constexpr int XPITCH = CIN1 * 2 + 16;      // 176
  constexpr int OPITCH = NCOL * 2 + 16;      // output staging
  constexpr int XPIECES = (XR * XPITCH + 1023) / 1024;
  constexpr int XPW = (XPIECES + NWV - 1) / NWV;
  constexpr int NU1 = (KS * CIN1 + 31) / 32;  // 13 flat units
  constexpr int NKS = NCOL / 32;              // 16 k-steps per tap (conv2)
  constexpr int NU2 = KS * NKS;               // 80
  constexpr int ZBYTES = NKS * 64;            // masked conv2 rows read base 0 + 64 ks (+16 hi)
  constexpr int Y_OFF = ZBYTES;
  constexpr int YREG = YR * YPITCH > BM * OPITCH ? YR * YPITCH : BM * OPITCH;
  constexpr int X_OFF = Y_OFF + YREG;
  constexpr int B1_OFF = X_OFF + NWV * XPW * 1024;
  constexpr int B2_OFF = B1_OFF + NCOL * 4;
  constexpr int SMEM = B2_OFF + NCOL * 4;
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M, T = p.T, pad = p.pad;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int hrow0 = lane & 15, hi = lane >> 4;
  auto taps = [&](int gm) {  // bit tap: row gm's tap stays inside its sequence
    int v = 0;
    if (gm >= 0 && gm < M) {
      int tpos, tlen;
      seq_pos(p.row_pos, gm, T, tpos, tlen);
#pragma unroll
      for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(tpos + tap - pad) < (unsigned)tlen ? 1 : 0) << tap;
    }
    return v;
  };
  for (int i = tid; i < ZBYTES / 16; i += NT) *reinterpret_cast<float4 *>(smem + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  // b1 | b2 -> LDS by LDS-DMA (waves 0..3, one 1 KiB piece each; B2_OFF = B1_OFF + 2 KiB)
  if (w < 4)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(w < 2 ? p.b1 : p.b2, NCOL * 4),
                                             (__attribute__((address_space(3))) void *)(smem + B1_OFF + w * 1024), 16,
                                             (uint32_t)((w & 1) * 1024 + lane * 16), 0, 0, 0);

  // mel tile -> LDS (lane-linear 1 KiB pieces at the padded pitch)
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const rsrc_t w1r = make_rsrc(p.w1, p.w1_bytes), w2r = make_rsrc(p.w2, p.w2_bytes);
  const uint32_t xrow = (uint32_t)p.xs * 2u;
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int pc = w + NWV * i;
    const int o = pc * 1024 + lane * 16;
    const int r = o / XPITCH, within = o - r * XPITCH;
    const int gm = m0 - 2 * pad + r;
    const bool ok = r < XR && within < CIN1 * 2 && gm >= 0 && gm < M;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                             16, ok ? (uint32_t)gm * xrow + (uint32_t)within : kOOB, 0, 0, 0);
  }

  // one weight stream per wave: units 0..12 of conv1 twice (two row passes), then conv2's 80
  const uint32_t lane_off = (uint32_t)lane * 16u;
  const uint32_t wb1 = (uint32_t)(w * NU1) * (uint32_t)kUnitB, wb2 = (uint32_t)(w * NU2) * (uint32_t)kUnitB;
  bf16x8 pa[DEPTH][JB];
  auto load_at = [&](auto S, int u) {  // u: position in the stream (past the end: a harmless reload)
    constexpr int s = decltype(S)::value;
    const bool c1 = u < 2 * NU1;
    const int uu = c1 ? (u < NU1 ? u : u - NU1) : (u - 2 * NU1 < NU2 ? u - 2 * NU1 : 0);
    const rsrc_t r = c1 ? w1r : w2r;
    const uint32_t so = (c1 ? wb1 : wb2) + (uint32_t)uu * (uint32_t)kUnitB;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jb = 0; jb < JB; ++jb)
      pa[s][jb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off + jb * 1024, so, 0));
    __builtin_amdgcn_sched_barrier(0);
  };
  static_for<DEPTH>([&](auto S) { load_at(S, decltype(S)::value); });
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * DEPTH) : "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();

  // ---- conv1 in two passes of 4 row blocks (y1 rows 0..63, 64..127; rows >= 116 are dropped)
  static_for<2>([&](auto PASS) {
    constexpr int ps = decltype(PASS)::value;
    int vm1[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) vm1[mb] = taps(m0 - pad + (4 * ps + mb) * 16 + hrow0);
    f32x4 acc[JB][4];
#pragma unroll
    for (int i = 0; i < JB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // flat unit u, lane group hi: k = 32u + 8hi -> (tap, channel); k >= 400: zero weights
    auto bases = [&](int u, int (&ad)[4]) {
      const int k = 32 * u + 8 * hi;
      const int tap = k / CIN1, c = k - tap * CIN1;
      const int base = X_OFF + ((4 * ps) * 16 + hrow0 + tap) * XPITCH + c * 2;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        ad[mb] = tap < KS ? (base + mb * 16 * XPITCH) & __builtin_amdgcn_sbfe(vm1[mb], tap, 1) : 0;
    };
    bf16x8 f0[4], f1[4];
    auto rd = [&](const int (&ad)[4], bf16x8 (&f)[4]) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) f[mb] = *reinterpret_cast<const bf16x8 *>(smem + ad[mb]);
    };
    int ad[4];
    bases(0, ad);
    rd(ad, f0);
    static_for<NU1>([&](auto UI) {
      constexpr int u = decltype(UI)::value, sl = (ps * NU1 + u) % DEPTH;
      if constexpr (u + 1 < NU1) {
        bases(u + 1, ad);
        if constexpr (u & 1) rd(ad, f0); else rd(ad, f1);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int jb = 0; jb < JB; ++jb)
          acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[sl][jb], (u & 1) ? f1[mb] : f0[mb], acc[jb][mb], 0, 0, 0);
      load_at(std::integral_constant<int, sl>{}, ps * NU1 + u + DEPTH);
    });
    // + b1, tanh, bf16 -> y1 rows (the conv2 x tile); rows past YR are not needed
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) {
      const int n = w * 64 + jb * 16 + 4 * hi;
      const float4 bb = *reinterpret_cast<const float4 *>(smem + B1_OFF + 4 * n);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int r = (4 * ps + mb) * 16 + hrow0;
        const f32x4 v = acc[jb][mb];
        bf16x4 o;
        o[0] = (bf16)tanh_fast(v[0] + bb.x);
        o[1] = (bf16)tanh_fast(v[1] + bb.y);
        o[2] = (bf16)tanh_fast(v[2] + bb.z);
        o[3] = (bf16)tanh_fast(v[3] + bb.w);
        if (r < YR) *reinterpret_cast<bf16x4 *>(smem + Y_OFF + r * YPITCH + n * 2) = o;
      }
    }
  });
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();  // y1 visible

  // ---- conv2 on the y1 tile (wconv's main loop)
  int vm2[MB];  // (computed here: kept live through conv1 they cost a spill)
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) vm2[mb] = taps(m0 + mb * 16 + hrow0);
  auto bases_x = [&](int tap, int (&ad)[MB]) {
    const int base = Y_OFF + (hrow0 + tap) * YPITCH + hi * 16;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) ad[mb] = (base + mb * 16 * YPITCH) & __builtin_amdgcn_sbfe(vm2[mb], tap, 1);
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
  constexpr int S0 = 2 * NU1;  // stream position of conv2's unit 0
  int bxc[MB], bxn[MB];
  bases_x(0, bxc);
  issue_x(bxc, std::integral_constant<int, 0>{}, f0);
#pragma nounroll
  for (int tap = 0; tap < KS; ++tap) {
    bases_x(tap + 1, bxn);  // tap KS: every row masked (zero region), a harmless read
    static_for<NKS>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value, sl = (S0 + ks) % DEPTH;
      if constexpr (ks + 1 < NKS) {
        if constexpr (ks & 1)
          issue_x(bxc, std::integral_constant<int, ks + 1>{}, f0);
        else
          issue_x(bxc, std::integral_constant<int, ks + 1>{}, f1);
      } else {
        issue_x(bxn, std::integral_constant<int, 0>{}, f0);
      }
      if constexpr (ks & 1)
        mma(pa[sl], f1);
      else
        mma(pa[sl], f0);
      load_at(std::integral_constant<int, sl>{}, S0 + tap * NKS + ks + DEPTH);
    });
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) bxc[mb] = bxn[mb];
  }

  // epilogue: + b2, tanh, bf16 -> LDS staging (the y1 region) -> whole-row stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();
#pragma unroll
  for (int nb = 0; nb < JB; ++nb) {
    const int n = w * 64 + nb * 16 + 4 * hi;
    const float4 bb = *reinterpret_cast<const float4 *>(smem + B2_OFF + 4 * n);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[nb][mb];
      bf16x4 o;
      o[0] = (bf16)tanh_fast(v[0] + bb.x);
      o[1] = (bf16)tanh_fast(v[1] + bb.y);
      o[2] = (bf16)tanh_fast(v[2] + bb.z);
      o[3] = (bf16)tanh_fast(v[3] + bb.w);
      *reinterpret_cast<bf16x4 *>(smem + Y_OFF + (hrow0 + mb * 16) * OPITCH + n * 2) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = NCOL * 2 / 16;
  char *ob = reinterpret_cast<char *>(p.out);
  const uint32_t orow = (uint32_t)p.os * 2u;
#pragma unroll 2
  for (int i = tid; i < BM * CPR; i += NT) {
    const int m = i / CPR, ch = i - m * CPR;
    if (m0 + m < M)
      store16_out(ob, (uint32_t)(m0 + m) * orow + (uint32_t)ch * 16u,
                  *reinterpret_cast<const uint4 *>(smem + Y_OFF + m * OPITCH + ch * 16), p.out_sc1);
  }
}


// The PostNet's last convolution + the residual (transformer/Layers.py:129-137, fastspeech2.py:136):
//   out[m, n] = sum_{tap, c} x[m + tap - 2, c] w[n, c, tap] + b[n] + res[m, n]     N = 80, Cin = 512
// N = 80 fills 62.5 % of a 128-wide tile (the conv_gemm launch: 40 us at cfg2, 0.11 of peak). Here
// the 80 output columns are 5 MFMA blocks that EVERY wave computes for its own rows: 4 waves x 2
// row blocks of the 112-row tile (the 8th block is a masked dummy), so the weights are shared
// by all waves and go through LDS: a 4-stage ring of k-steps (5 x 1 KiB fragment-ordered blocks,
// LDS-DMA, one counted vmcnt + barrier per k-step), the x tile DMA'd once as in wconv. Per k-step
// and wave: 5 + 2 fragment reads, 10 MFMAs. f32 out through an LDS staging tile (whole rows).
struct PnTailArgs {
  const bf16 *x;
  int64_t xs;
  const bf16 *w;  // [80 k-steps][5 blocks][4][16][8]
  const float *bias;
  const float *res;
  int64_t rs;
  float *out;
  int64_t os;
  int T, M, pad;
  uint32_t x_bytes, w_bytes;
  const int2 *row_pos;
  const int32_t *rows_dev;
};

__global__ __launch_bounds__(256, 1) void pn_tail_kernel(PnTailArgs p) {
  constexpr int KS = 5, CIN = 512, NB = 5, NCOL = 80, BM = 112, NST = 3, KPS = 2;
  constexpr int XR = BM + KS - 1;
  constexpr int XPITCH = CIN * 2 + 32;
  constexpr int XPIECES = (XR * XPITCH + 1023) / 1024;
  constexpr int XPW = (XPIECES + 3) / 4;
  constexpr int NKS = CIN / 32, NU = KS * NKS;  // 16 k-steps per tap, 80 in all
  constexpr int NS = NU / KPS;                  // ring stages of 2 k-steps
  constexpr int PPS = 12;                       // 10 weight pieces + 2 dummies: every wave issues 3
  constexpr int STG = PPS * 1024;
  constexpr int ZBYTES = NKS * 64;
  constexpr int X_OFF = ZBYTES;
  constexpr int W_OFF = X_OFF + 4 * XPW * 1024;
  constexpr int B_OFF = W_OFF + NST * STG;
  constexpr int SMEM = B_OFF + NCOL * 4;
  constexpr int OPITCH = NCOL * 4 + 16;         // f32 staging (in the x region)
  static_assert(BM * OPITCH <= 4 * XPW * 1024, "staging fits the x region");
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M, T = p.T, pad = p.pad;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int hrow0 = lane & 15, hi = lane >> 4;
  int vm[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rb = 2 * w + j;
    const int m = m0 + rb * 16 + hrow0;
    int v = 0;
    if (rb * 16 < BM && m < M) {
      int tpos, tlen;
      seq_pos(p.row_pos, m, T, tpos, tlen);
#pragma unroll
      for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(tpos + tap - pad) < (unsigned)tlen ? 1 : 0) << tap;
    }
    vm[j] = v;
  }
  for (int i = tid; i < ZBYTES / 16; i += 256) *reinterpret_cast<float4 *>(smem + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < NCOL / 4)
    *reinterpret_cast<float4 *>(smem + B_OFF + 16 * tid) = reinterpret_cast<const float4 *>(p.bias)[tid];

  const rsrc_t xr = make_rsrc(p.x, p.x_bytes), wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t xrow = (uint32_t)p.xs * 2u;
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int pc = w + 4 * i;
    const int o = pc * 1024 + lane * 16;
    const int r = o / XPITCH, within = o - r * XPITCH;
    const int gm = m0 - pad + r;
    const bool ok = r < XR && within < CIN * 2 && gm >= 0 && gm < M;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + X_OFF + pc * 1024),
                                             16, ok ? (uint32_t)gm * xrow + (uint32_t)within : kOOB, 0, 0, 0);
  }
  // stage s (k-steps 2s, 2s + 1) -> ring slot s % NST: wave w DMAs pieces w, w + 4, w + 8 (pieces
  // 10, 11: dummies, zeros)
  auto wdma = [&](int st_idx) {
    char *st = smem + W_OFF + (st_idx % NST) * STG;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int pc = w + 4 * j;
      const uint32_t off = pc < KPS * NB ? (uint32_t)(st_idx * KPS * NB + pc) * 1024u + (uint32_t)lane * 16u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(st + pc * 1024), 16, off,
                                               0, 0, 0);
    }
  };
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) wdma(st);

  f32x4 acc[NB][2];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b][0] = acc[b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // stage s: k-steps u = 2s + q (tap = u / 16): every fragment read first, then the 20 MFMAs
  auto stage = [&](int st_idx) {
    const char *st = smem + W_OFF + (st_idx % NST) * STG;
    bf16x8 fa[KPS][NB], fb[KPS][2];
#pragma unroll
    for (int q = 0; q < KPS; ++q) {
      const int u = st_idx * KPS + q, tap = u >> 4, ks = u & 15;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ad = (X_OFF + ((2 * w + j) * 16 + hrow0 + tap) * XPITCH + hi * 16) & __builtin_amdgcn_sbfe(vm[j], tap, 1);
        fb[q][j] = *reinterpret_cast<const bf16x8 *>(smem + ad + ks * 64);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) fa[q][b] = *reinterpret_cast<const bf16x8 *>(st + (q * NB + b) * 1024 + lane * 16);
    }
#pragma unroll
    for (int q = 0; q < KPS; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q][b], fb[q][j], acc[b][j], 0, 0, 0);
  };
  // the x tile (issued first) and stage 0 landed; stage 1 may stay in flight
  asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();
#pragma nounroll
  for (int st = 0; st < NS; ++st) {
    if (st > 0) {
      // stage st landed (this wave's pieces; the next stage may stay in flight) and visible to all
      // waves; every wave is past stage st - 1, whose slot the DMA below refills
      if (st + 1 < NS)
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (st + NST - 1 < NS) wdma(st + NST - 1);
    stage(st);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __syncthreads();  // every wave is done with the x tile: it becomes the f32 staging tile
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int n = b * 16 + 4 * hi;
    const float4 bb = *reinterpret_cast<const float4 *>(smem + B_OFF + 4 * n);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = (2 * w + j) * 16 + hrow0;
      if (r < BM) {
        const f32x4 v = acc[b][j];
        *reinterpret_cast<float4 *>(smem + X_OFF + r * OPITCH + n * 4) =
            make_float4(v[0] + bb.x, v[1] + bb.y, v[2] + bb.z, v[3] + bb.w);
      }
    }
  }
  __syncthreads();
  constexpr int CPR = NCOL * 4 / 16;  // 20 16-byte chunks per row
  for (int i = tid; i < BM * CPR; i += 256) {
    const int m = i / CPR, ch = i - m * CPR;
    if (m0 + m < M) {
      const float4 a = *reinterpret_cast<const float4 *>(smem + X_OFF + m * OPITCH + ch * 16);
      const float4 r = *reinterpret_cast<const float4 *>(p.res + (size_t)(m0 + m) * p.rs + ch * 4);
      *reinterpret_cast<float4 *>(p.out + (size_t)(m0 + m) * p.os + ch * 4) =
          make_float4(a.x + r.x, a.y + r.y, a.z + r.z, a.w + r.w);
    }
  }
}

}  // namespace

extern "C" int64_t fs2_wconv_weight_elems(int KS, int Cin, int N) { return (int64_t)N * ((KS * Cin + 31) / 32 * 32); }

extern "C" int fs2_wconv(const fs2_wconv_desc *d, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->bias == nullptr || d->out == nullptr)
    return FS2_EINVAL;
  const bool fused_tail = d->w2 != nullptr && d->Cin == 512;  // out: the f32 [B*T, 80] tail output
  if (d->B < 0 || d->T < 0 || d->pad < 0 || d->x_row_stride < d->Cin || (d->x_row_stride & 7) ||
      (!fused_tail && (d->out_row_stride < d->N || (d->out_row_stride & 7))))
    return FS2_EINVAL;
  const bool tail = d->epilogue == FS2_EPI_BIAS_RES;  // the last conv: N = 80, + residual, f32 out
  if (tail) {
    if (d->Cin != 512 || d->N != 80 || d->KS != 5 || d->pad != 2 || d->w2 != nullptr) return FS2_EUNSUPPORTED;
    if (d->residual == nullptr || d->res_row_stride < 80 || (d->res_row_stride & 3) || (d->out_row_stride & 3))
      return FS2_EINVAL;
  } else if (!(d->Cin == 512 || d->Cin == 80) || d->N != 512 || d->KS != 5 || d->pad > d->KS - 1 ||
             d->epilogue != FS2_EPI_BIAS_TANH) {
    return FS2_EUNSUPPORTED;
  }
  if (d->x == d->out) return FS2_EINVAL;  // other tiles re-read x rows (halo)
  if ((d->rows_dev == nullptr) != (d->row_pos == nullptr)) return FS2_EINVAL;
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 == 0) return FS2_OK;
  const int64_t xb = M64 * d->x_row_stride * 2;
  if (xb >= (1LL << 31) || M64 > 0x7fffff00LL) return FS2_EUNSUPPORTED;
  const int2 *row_pos = reinterpret_cast<const int2 *>(d->row_pos);
  // packed rows: the grid covers rows_max (the host's bound on the device row count) when given
  const int64_t Mg = (d->rows_dev != nullptr && d->rows_max > 0 && d->rows_max < M64) ? d->rows_max : M64;
  if (tail) {
    PnTailArgs q;
    q.x = reinterpret_cast<const bf16 *>(d->x);
    q.xs = d->x_row_stride;
    q.w = reinterpret_cast<const bf16 *>(d->w);
    q.bias = d->bias;
    q.res = d->residual;
    q.rs = d->res_row_stride;
    q.out = reinterpret_cast<float *>(d->out);
    q.os = d->out_row_stride;
    q.T = d->T;
    q.M = (int)M64;
    q.pad = d->pad;
    q.x_bytes = (uint32_t)xb;
    q.w_bytes = (uint32_t)(fs2_wconv_weight_elems(d->KS, d->Cin, d->N) * 2);
    q.row_pos = row_pos;
    q.rows_dev = d->rows_dev;
    q.M = (int)Mg;
    hipLaunchKernelGGL(pn_tail_kernel, dim3((unsigned)((Mg + 111) / 112)), dim3(256), 0, as_stream(stream), q);
    FS2_CHECK_LAUNCH();
    return FS2_OK;
  }
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
  p.row_pos = row_pos;
  p.rows_dev = d->rows_dev;
  p.M = (int)Mg;
  p.out_sc1 = env_out_sc1();
  const int nwg = (int)((Mg + 111) / 112);
#ifndef WCONV_WQ
#define WCONV_WQ 1  // 8 waves x 64 columns (2 quads per wave: 224 accumulators + the ring spill; analysis only)
#endif
  if (fused_tail) {
    // the PostNet's last two layers fused (512 -> 512 tanh, then 512 -> 80 + residual, f32 out)
    if (d->bias2 == nullptr || d->residual == nullptr || d->pad != 2 || d->res_row_stride < 80 ||
        (d->res_row_stride & 3) || d->out_row_stride < 80 || (d->out_row_stride & 3))
      return FS2_EINVAL;
    p.w2 = reinterpret_cast<const bf16 *>(d->w2);
    p.bias2 = d->bias2;
    p.res = d->residual;
    p.rs = d->res_row_stride;
    p.out2 = reinterpret_cast<float *>(d->out);
    p.os2 = d->out_row_stride;
    p.out = nullptr;
    p.w2_bytes = (uint32_t)(fs2_wconv_weight_elems(5, 512, 80) * 2);
    hipLaunchKernelGGL((wconv_kernel<5, 512, 1, true>), dim3((unsigned)((Mg + 107) / 108)), dim3(512), 0,
                       as_stream(stream), p);
  } else if (d->w2 != nullptr) {
    // the PostNet's first two layers fused (80 -> 512 -> 512, both tanh)
    if (d->Cin != 80 || d->bias2 == nullptr || d->pad != 2) return FS2_EUNSUPPORTED;
    PnHeadArgs q;
    q.x = p.x;
    q.xs = p.xs;
    q.w1 = p.w;
    q.w2 = reinterpret_cast<const bf16 *>(d->w2);
    q.b1 = d->bias;
    q.b2 = d->bias2;
    q.out = p.out;
    q.os = p.os;
    q.T = p.T;
    q.M = p.M;
    q.pad = p.pad;
    q.x_bytes = p.x_bytes;
    q.w1_bytes = p.w_bytes;
    q.w2_bytes = (uint32_t)(fs2_wconv_weight_elems(d->KS, 512, 512) * 2);
    q.row_pos = row_pos;
    q.rows_dev = d->rows_dev;
    q.out_sc1 = env_out_sc1();
    hipLaunchKernelGGL(pn_head_kernel, dim3(nwg), dim3(512), 0, as_stream(stream), q);
  } else if (d->Cin == 80)
    hipLaunchKernelGGL((wconv_kernel<5, 80, 1>), dim3(nwg), dim3(512), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((wconv_kernel<5, 512, WCONV_WQ>), dim3(nwg), dim3(512 / WCONV_WQ), 0, as_stream(stream), p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
