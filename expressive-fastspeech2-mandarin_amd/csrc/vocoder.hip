// HiFi-GAN V1 multi-receptive-field fusion (hifigan/models.py:20-45 ResBlock1 + :152-158) as ONE
// kernel per upsampling stage, for the narrow late stages (C = 64, 32 channels):
//
//   xs = sum_{k in (3, 7, 11)} ResBlock_k(x);   out = leaky_relu(xs / 3, slope)
//   ResBlock_k(x): for d in (1, 3, 5):  x = conv_k,1(lrelu(conv_k,d(lrelu(x)) + b1)) + b2 + x
//
// As 18 separate conv launches per stage each conv read and wrote a [B, T*128 or *256, C] tensor
// (451 MB at cfg2) with C = 32 / 64 filling an MFMA tile's N side a quarter / half: stages 3 and 4
// took 11.2 and 15.5 ms of a 43 ms vocoder call. Here a workgroup owns L = 256 output samples of
// one utterance and runs all 18 convs on chip: the input tile with a 64-sample halo (each k chain
// reaches 6 (k - 1) <= 60 samples) is DMA'd to LDS, the chains' intermediates never leave the CU,
// and only lrelu(xs / 3) is written (the next upsampler's / conv_post's input).
//
// * Conv step = implicit GEMM D[ch][row] = sum_{tap, c} W[ch][c][tap] . IN[row + (tap - hk) d][c]:
//   weights are the MFMA A operand (16-channel blocks, fragment-ordered, read from L2/L1 one k-step
//   ahead), activations the B operand from LDS; output rows in 16-row blocks dealt round-robin to
//   the 4 waves. Each step computes only the rows later steps need (the halo shrinks along the chain).
// * LDS: three [384 rows x C] bf16 buffers -- CUR (the chain's running x), ACT (lrelu(CUR)), T
//   (lrelu(conv1 + b1)) -- with a row XOR swizzle on the 16-byte chunk (found by exhaustive search:
//   the 16 rows x 16 bytes of a fragment read are conflict-free for any tap shift).
// * Sequence edges: rows outside [0, T) are written as zeros after every step (nn.Conv1d's zero
//   padding); the chains' sums xs stay in f32 registers (the last conv of each chain produces the
//   same rows on the same waves).
#include <type_traits>
#include <utility>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

constexpr int kMrfL = 256;              // output samples per workgroup
constexpr int kMrfH = 64;               // halo rows each side (>= 6 (11 - 1) = 60)
constexpr int kMrfR = kMrfL + 2 * kMrfH;  // 384 buffer rows
constexpr int kMrfNB = kMrfR / 16;      // 24 row blocks
constexpr int kMrfLgkm0 = 0xC07F;

struct MrfArgs {
  const bf16 *x;     // ups output [B, T, C]
  const bf16 *a0;    // lrelu(x) [B, T, C] (the ups epilogue's second output)
  const bf16 *w;     // 18 convs, fragment order (see mrf_woff)
  const float *bias; // [18][C]
  bf16 *out;         // lrelu(xs / 3, slope) [B, T, C]
  int T, ntiles;     // samples per utterance, tiles per utterance
  float slope;       // output leaky_relu slope (0.1 before an upsampler, 0.01 before conv_post)
  uint32_t x_bytes;
};

template <typename Fn, int... I>
__device__ __forceinline__ void mrf_static_for_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void mrf_static_for(Fn &&f) {
  mrf_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// chunk swizzle of a C-channel bf16 row (C / 8 chunks of 16 bytes)
template <int C>
__device__ __forceinline__ int mrf_swz(int r) {
  if constexpr (C == 32) return (r & 4) ? 2 : 0;
  else return ((r & 2) ? 2 : 0) ^ ((r & 4) ? 4 : 0);
}

__device__ __forceinline__ float lrelu(float v, float s) { return v > 0.f ? v : v * s; }

// element offset of conv (chain j, pair p, second) in the packed weights: per conv [k * C/32 k-steps]
// [C/16 blocks][64 lanes][8]
template <int C>
__host__ __device__ constexpr int mrf_conv_elems(int k) { return k * C * C; }
template <int C>
__host__ __device__ constexpr int mrf_woff(int j, int p, int second) {
  int off = 0;
  const int ks[3] = {3, 7, 11};
  for (int jj = 0; jj < j; ++jj) off += 6 * mrf_conv_elems<C>(ks[jj]);
  return off + (2 * p + second) * mrf_conv_elems<C>(ks[j]);
}

// NW waves: 4 for C = 32 (two workgroups per CU fit LDS), 8 for C = 64 (one workgroup per CU:
// two waves per SIMD hide the LDS / weight latency a single wave exposed)
template <int C, int NW>
__global__ __launch_bounds__(64 * NW) void mrf_kernel(MrfArgs p) {
  constexpr int kMrfNBW = kMrfNB / NW;  // row blocks per wave
  constexpr int NXS = 16 / NW;          // output row blocks (4..19) per wave
  constexpr int RB = C * 2;          // row bytes
  constexpr int NCB = C / 16;        // channel blocks (MFMA A blocks)
  constexpr int KC = C / 32;         // 32-channel k-steps per tap
  constexpr int BUF = kMrfR * RB;
  constexpr int CUR_OFF = 0, ACT_OFF = BUF, T_OFF = 2 * BUF;
  constexpr int SMEM = 3 * BUF;
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int utt = blockIdx.y, tile = blockIdx.x;
  const int T = p.T;
  const int t0 = tile * kMrfL - kMrfH;  // global sample of buffer row 0
  const int64_t ubase = (int64_t)utt * T;
  const int r16 = lane & 15, g = lane >> 4;

  // buffer row R holds sample t0 + R: inside the utterance?
  auto inside = [&](int R) __attribute__((always_inline)) { return (unsigned)(t0 + R) < (unsigned)T; };

  // ---- DMA of the chain input: CUR <- x, ACT <- lrelu(x) (rows outside [0, T): zeros)
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes), ar = make_rsrc(p.a0, p.x_bytes);
  auto load_input = [&]() __attribute__((always_inline)) {
    constexpr int RPP = 1024 / RB;  // rows per 1 KiB piece
    constexpr int NP = BUF / 1024;
#pragma unroll
    for (int i = 0; i < (NP + NW - 1) / NW; ++i) {
      const int pc = w + NW * i;
      if (pc < NP) {
        const int R = pc * RPP + lane / (RB / 16), phys = lane % (RB / 16);
        const int logical = phys ^ mrf_swz<C>(R);
        const uint32_t off = inside(R) ? (uint32_t)((ubase + t0 + R) * RB + logical * 16) : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + CUR_OFF + pc * 1024),
                                                 16, off, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, (__attribute__((address_space(3))) void *)(smem + ACT_OFF + pc * 1024),
                                                 16, off, 0, 0, 0);
      }
    }
  };
  auto sync = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // LDS byte address of (row R, 8-channel group q)
  auto addr = [&](int buf, int R, int q) __attribute__((always_inline)) {
    return buf + R * RB + ((q ^ mrf_swz<C>(R)) << 4);
  };

  f32x4 xs[NXS][NCB];  // the chains' sum over output rows [64, 320): blocks b = w (mod NW)
#pragma unroll
  for (int i = 0; i < NXS; ++i)
#pragma unroll
    for (int c = 0; c < NCB; ++c) xs[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one conv step: output blocks [blo, bhi), kernel K (taps), dilation D, input buffer IN;
  // kind 0: T = lrelu(acc + b) ; 1: CUR = acc + b + CUR, ACT = lrelu(CUR) ; 2: xs += acc + b + CUR
  // (every lambda is force-inlined: an out-of-line call kept acc / xs on the scratch stack)
  auto step = [&](int kind, int K, int D, int IN, const bf16 *wc, const float *bc, int blo,
                  int bhi) __attribute__((always_inline)) {
    const int hk = (K - 1) / 2;
    const rsrc_t wr = make_rsrc(wc, (uint32_t)(K * C * C * 2));
    f32x4 acc[kMrfNBW][NCB];
#pragma unroll
    for (int i = 0; i < kMrfNBW; ++i)
#pragma unroll
      for (int c = 0; c < NCB; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int first = blo + ((w - blo) % NW + NW) % NW;  // this wave's first block (b = w mod NW)
    const int nks = K * KC;
    bf16x8 wa[2][NCB];
    auto wload = [&](int s, bf16x8 (&f)[NCB]) __attribute__((always_inline)) {
#pragma unroll
      for (int c = 0; c < NCB; ++c)
        f[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              wr, (uint32_t)lane * 16u, (uint32_t)((s * NCB + c) * 1024), 0));
    };
    // k-step s with its weights in wc (loaded one step ahead into wn)
    auto kstep = [&](int s, const bf16x8 (&wc)[NCB], bf16x8 (&wn)[NCB]) __attribute__((always_inline)) {
      if (s + 1 < nks) {
        wload(s + 1, wn);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NCB) : "memory");  // this k-step's weights (the next may fly)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const int tap = s / KC, kc = s - tap * KC;
      const int shift = (tap - hk) * D;
#pragma unroll
      for (int i = 0; i < kMrfNBW; ++i) {
        const int b = first + NW * i;
        if (b < bhi) {  // wave-uniform
          const int R = min(max(b * 16 + r16 + shift, 0), kMrfR - 1);
          const bf16x8 fb = *reinterpret_cast<const bf16x8 *>(smem + addr(IN, R, 4 * kc + g));
#pragma unroll
          for (int c = 0; c < NCB; ++c)
            acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc[c], fb, acc[i][c], 0, 0, 0);
        }
      }
    };
    if constexpr (C == 32) {
      // 32 channels: a k-step is only 12 MFMAs per wave, shorter than an L2 round trip, so the
      // whole conv's weights (<= 11 k-steps x 2 fragments = 88 VGPRs) are loaded up front and the
      // latency is paid once per conv instead of once per k-step
      bf16x8 wall[11][NCB];
#pragma unroll
      for (int st = 0; st < 11; ++st)
        if (st < nks) wload(st, wall[st]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int st = 0; st < 11; ++st) {
        if (st < nks) {
          const int shift = (st - hk) * D;  // KC == 1: k-step = tap
#pragma unroll
          for (int i = 0; i < kMrfNBW; ++i) {
            const int b = first + NW * i;
            if (b < bhi) {
              const int R = min(max(b * 16 + r16 + shift, 0), kMrfR - 1);
              const bf16x8 fb = *reinterpret_cast<const bf16x8 *>(smem + addr(IN, R, g));
#pragma unroll
              for (int c = 0; c < NCB; ++c)
                acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wall[st][c], fb, acc[i][c], 0, 0, 0);
            }
          }
        }
      }
    } else {
      wload(0, wa[0]);
      int s = 0;
      for (; s + 1 < nks; s += 2) {
        kstep(s, wa[0], wa[1]);
        kstep(s + 1, wa[1], wa[0]);
      }
      if (s < nks) kstep(s, wa[0], wa[1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
    __builtin_amdgcn_s_barrier();  // every wave done reading IN (and T may be rewritten)
    // epilogue: lane holds channels 16c + 4g .. +3 of row 16b + r16
#pragma unroll
    for (int i = 0; i < kMrfNBW; ++i) {
      const int b = first + NW * i;
      if (b < bhi) {
        const int R = b * 16 + r16;
        const bool in = inside(R);
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          const int ch = 16 * c + 4 * g;
          const float4 bb = *reinterpret_cast<const float4 *>(bc + ch);
          f32x4 v = acc[i][c];
          v[0] += bb.x;
          v[1] += bb.y;
          v[2] += bb.z;
          v[3] += bb.w;
          const int o = R * RB + (((ch >> 3) ^ mrf_swz<C>(R)) << 4) + (ch & 7) * 2;
          if (kind == 0) {
            bf16x4 t;
#pragma unroll
            for (int q = 0; q < 4; ++q) t[q] = (bf16)(in ? lrelu(v[q], 0.1f) : 0.f);
            *reinterpret_cast<bf16x4 *>(smem + T_OFF + o) = t;
          } else {
            const bf16x4 xo = *reinterpret_cast<const bf16x4 *>(smem + CUR_OFF + o);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] += (float)xo[q];
            if (kind == 1) {
              bf16x4 nc, na;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                nc[q] = (bf16)(in ? v[q] : 0.f);
                na[q] = (bf16)(in ? lrelu(v[q], 0.1f) : 0.f);
              }
              *reinterpret_cast<bf16x4 *>(smem + CUR_OFF + o) = nc;
              *reinterpret_cast<bf16x4 *>(smem + ACT_OFF + o) = na;
            } else if (i < NXS) {
              xs[i % NXS][c] += v;  // the last conv of a chain: its output blocks 4..19, rows 64..319
            }
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
    __builtin_amdgcn_s_barrier();  // the step's output visible
  };

  // runtime loops over the 3 chains x 3 dilation pairs x 2 convs: ONE inlined copy of the step code
  // (18 unrolled copies overflowed the instruction cache)
#pragma nounroll
  for (int j = 0; j < 3; ++j) {
    const int K = 3 + 4 * j, hk = (K - 1) / 2;
    load_input();
    sync();
#pragma nounroll
    for (int pp = 0; pp < 3; ++pp) {
      // rows each step must produce: [64 - e, 320 + e) with e = 11hk, 10hk, 7hk, 6hk, hk, 0
      const int e1 = pp == 0 ? 11 * hk : (pp == 1 ? 7 * hk : hk);
      const int e2 = pp == 0 ? 10 * hk : (pp == 1 ? 6 * hk : 0);
      const int dil = 1 + 2 * pp;
#pragma nounroll
      for (int half = 0; half < 2; ++half) {
        const int e = half == 0 ? e1 : e2;
        const int lo = (kMrfH - e) / 16, hi = (kMrfH + kMrfL + e + 15) / 16;
        const int kind = half == 0 ? 0 : (pp < 2 ? 1 : 2);
        step(kind, K, half == 0 ? dil : 1, half == 0 ? ACT_OFF : T_OFF, p.w + mrf_woff<C>(j, pp, half),
             p.bias + (j * 6 + 2 * pp + half) * C, lo, hi);
      }
    }
  }

  // ---- out = lrelu(xs / 3, slope) over the tile's 256 samples (blocks 4..19, NXS per wave)
#pragma unroll
  for (int i = 0; i < NXS; ++i) {
    const int b = 4 + ((w - 4) % NW + NW) % NW + NW * i;
    const int R = b * 16 + r16, t = t0 + R;
    if (t < T) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const f32x4 v = xs[i][c];
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)lrelu(v[q] * (1.0f / 3.0f), p.slope);
        *reinterpret_cast<bf16x4 *>(p.out + (ubase + t) * C + 16 * c + 4 * g) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// One ResBlock1 dilation pair at C = 128 (the 64x stage: 128 channels, T * 64 samples) in ONE
// launch (hifigan/models.py:34-45):
//
//   y = conv_k,1(lrelu(conv_k,d(lrelu(x)) + b1, 0.1)) + b2 + x (+ xs)
//   out = y, or lrelu(y * out_scale, out_slope) for the stage's last pair
//
// The whole-stage MRF form above needs three [384 x C] buffers (288 KiB at C = 128); as two conv
// launches per pair every intermediate made an HBM round trip (conv1 wrote t, conv2 read t and x
// and wrote x and lrelu(x): 2.7 GB per pair at cfg2, 12.4 ms of a 29.4 ms vocoder call). Here a
// workgroup owns L = 256 samples of one utterance:
// * A: lrelu(x) over [t0 - hk (D + 1), t0 + L + hk (D + 1)) by LDS-DMA + an in-place leaky_relu
//   (each lane converts the 16-byte chunks its own DMA wrote, after its own vmcnt wait);
// * T: lrelu(conv1 + b1) over [t0 - hk, t0 + L + hk) (17 row blocks), zeros outside [0, T);
// * conv2 over T, + b2 + x (registers, loaded at the start) (+ xs), staged in T's rows and stored
//   as whole 256-byte rows.
// 8 waves (two per SIMD), wave w owns output channels 16w .. 16w + 15 of both convs and every row
// block: its weight fragment of a k-step (1 KiB, fragment order of pack_wconv_tail) comes from
// L2 three k-steps ahead; the activations are the B operand from LDS. Rows are 256 B with the
// 16-byte chunk rotated by 2 * row (phys = (c + 2 r) & 15): the ds_read_b128 lane groups
// {0-3,12-15,20-27}, ... hit 16 distinct slots for every row shift (the bank behaviour of a
// 288-byte pitch, without its padding), and a 1 KiB LDS-DMA piece stays 4 whole rows.
constexpr int kPrNW = 8;  // waves

// per channel count: C = 128 (256-sample tiles, 256-byte rows, chunk rotated by 2 r) or C = 64
// (512-sample tiles, 128-byte rows, chunk rotated by r: the same ds_read_b128 lane-group check,
// two rows per 256-byte bank row)
template <int C>
struct PairCfg {
  static constexpr int L = C == 128 ? 256 : 512;  // output samples per workgroup
  static constexpr int RB = 2 * C;                // row bytes
  static constexpr int NCK = C / 8;               // 16-byte chunks per row
  static constexpr int NBT = L / 16 + 1;          // conv1 output row blocks (>= (L + 2 hk) / 16, k <= 11)
  static constexpr int NCP = C / 32;              // channel pairs (two 16-channel MFMA blocks each)
  static constexpr int NRG = kPrNW / NCP;         // row groups
  static constexpr int NB1 = (NBT + NRG - 1) / NRG;  // conv1 blocks per wave (the last group's extras dropped)
  static constexpr int NB2 = L / 16 / NRG;        // conv2 blocks per wave
  static constexpr int KC = C / 32;               // k-steps per tap
  __device__ static __forceinline__ int phys(int r, int c) {
    return C == 128 ? (c + 2 * r) & 15 : (c + r) & 7;
  }
};

struct PairArgs {
  const bf16 *x;        // [B, T, C] pair input (residual; conv1 reads lrelu(x))
  const bf16 *w1, *w2;  // pack_wconv_tail fragment order, [k * C/32 k-steps][C/16 blocks][64][8]
  const float *b1, *b2; // [C]
  const bf16 *xs;       // optional running sum (may alias out)
  bf16 *out;            // [B, T, C]
  int T, D;             // samples per utterance, conv1 dilation
  float out_scale, out_slope;
  int out_act;          // 0: out = y; 1: out = lrelu(y * out_scale, out_slope)
  uint32_t x_bytes;
};

template <int C, int K>
__global__ __launch_bounds__(64 * kPrNW) void pair_kernel(PairArgs p) {
  using Q = PairCfg<C>;
  constexpr int L = Q::L, RB = Q::RB, NCK = Q::NCK, NBT = Q::NBT, NB1 = Q::NB1, NB2 = Q::NB2, KC = Q::KC;
  constexpr int HK = (K - 1) / 2;
  // A rows: L + 2 hk (D + 1) <= L + 12 hk (D <= 5), rounded to whole 1 KiB pieces, + the rows the
  // dropped conv1 blocks and the unused output rows (>= L + 2 hk) read past them (stale data there
  // reaches only those rows)
  constexpr int RPP = 1024 / RB;  // rows per DMA piece
  constexpr int RA_MAX = L + 12 * HK + RPP + 16 * (NB1 * Q::NRG - NBT) + 16;
  constexpr int A_OFF = 0, T_OFF = RA_MAX * RB;
  constexpr int SMEM = T_OFF + NBT * 16 * RB;
  static_assert(SMEM <= 163840, "LDS");
  static_assert(L + 2 * HK <= NBT * 16, "conv1 rows");
  static_assert(16 * NB2 * Q::NRG == L, "conv2 rows");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int T = p.T, D = p.D;
  const int t0 = blockIdx.x * L;
  const int64_t ubase = (int64_t)blockIdx.y * T;
  const int HA = HK * (D + 1);         // A halo
  const int RA = L + 2 * HA;           // A rows of this launch
  const int a0 = t0 - HA;              // sample of A row 0
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);

  // ---- A <- x over [a0, a0 + RA) (whole pieces) by LDS-DMA (rows outside [0, T) read as zeros)
  const int npc = (RA + RPP - 1) / RPP;  // 1 KiB pieces
  for (int pc = w; pc < npc; pc += kPrNW) {
    const int R = RPP * pc + lane / NCK, ph = lane % NCK;
    const int c = C == 128 ? (ph - 2 * R) & 15 : (ph - R) & 7, s = a0 + R;
    const uint32_t off = (unsigned)s < (unsigned)T ? (uint32_t)((ubase + s) * RB + c * 16) : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(smem + A_OFF + pc * 1024),
                                             16, off, 0, 0, 0);
  }
  // wave w: output channels 32 cp .. 32 cp + 31 (two 16-channel MFMA blocks) of row group rg:
  // conv1 blocks NB1 rg .. +NB1-1, conv2 blocks NB2 rg .. +NB2-1. Every B fragment read from LDS
  // feeds two MFMAs (one wave per 16 channels over every row block read as many LDS cycles per
  // k-step as the MFMAs took)
  const int cp = w % Q::NCP, rg = w / Q::NCP;
  // the residual x of this wave's conv2 output (rows t0 + 16 (NB2 rg + b) + r16, channels
  // 32 cp + 16 j + 4 g .. +3)
  bf16x4 res[2][NB2];
#pragma unroll
  for (int b = 0; b < NB2; ++b) {
    const int s = t0 + 16 * (NB2 * rg + b) + r16;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t off = s < T ? (uint32_t)((ubase + s) * RB + (32 * cp + 16 * j + 4 * g) * 2) : kOOB;
      res[j][b] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // lrelu in place over this wave's own pieces
  for (int pc = w; pc < npc; pc += kPrNW) {
    bf16x8 *q = reinterpret_cast<bf16x8 *>(smem + A_OFF + pc * 1024 + lane * 16);
    bf16x8 v = *q;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16)lrelu((float)v[i], 0.1f);
    *q = v;
  }
  __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
  __builtin_amdgcn_s_barrier();

  // ---- one conv: NB row blocks from block b0 of IN, k-step s = tap * KC + kc, weights wp (blocks
  // 2 cp, 2 cp + 1), B row of output row r and tap: r + tap * dil (IN row; inside the A / T
  // regions by RA_MAX / NBT). A 4-slot register ring of weight pairs, loads 3 k-steps ahead: at
  // KC = 2 the tap loop walks tap pairs so every slot stays a constant.
  auto conv = [&](auto nb_tag, const bf16 *wp, int IN, int b0, int dil,
                  f32x4 (&acc)[2][decltype(nb_tag)::value]) __attribute__((always_inline)) {
    constexpr int NB = decltype(nb_tag)::value;
    constexpr int NKS = K * KC;
    const rsrc_t wr = make_rsrc(wp, (uint32_t)(K * C * C * 2));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[j][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 wf[4][2];
    auto wload = [&](int s, bf16x8 (&f)[2]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        f[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              wr, (uint32_t)lane * 16u, (uint32_t)((s * (C / 16) + 2 * cp + j) * 1024), 0));
    };
    // k-step s (ring slot SL = s & 3) of tap `tap`, channel step kc
    auto kstep = [&](auto sl_tag, int s, int tap, int kc) __attribute__((always_inline)) {
      constexpr int SL = decltype(sl_tag)::value;
      if (s + 3 < NKS) {
        wload(s + 3, wf[(SL + 3) & 3]);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // row 16 (b0 + b) + r16 + sh: the chunk rotation does not depend on b (16 rows shift it by
      // a multiple of the row's chunk count), so every block's read is one base + an immediate
      const int R0 = 16 * b0 + r16 + tap * dil;
      const char *base = smem + IN + R0 * RB + Q::phys(R0, 4 * kc + g) * 16;
      bf16x8 fb[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[b] = *reinterpret_cast<const bf16x8 *>(base + b * 16 * RB);
      // all reads issued before the first MFMA (interleaved read -> wait -> MFMA pairs exposed
      // the LDS latency on every MFMA)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[SL][j], fb[b], acc[j][b], 0, 0, 0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    wload(0, wf[0]);
    wload(1, wf[1]);
    wload(2, wf[2]);
    if constexpr (KC == 4) {
#pragma nounroll
      for (int tap = 0; tap < K; ++tap) {
        kstep(I0{}, 4 * tap, tap, 0);
        kstep(I1{}, 4 * tap + 1, tap, 1);
        kstep(I2{}, 4 * tap + 2, tap, 2);
        kstep(I3{}, 4 * tap + 3, tap, 3);
      }
    } else {
      static_assert(KC == 2 && (K & 1), "tap pairs + one tap");
#pragma nounroll
      for (int tap = 0; tap + 1 < K; tap += 2) {
        kstep(I0{}, 2 * tap, tap, 0);
        kstep(I1{}, 2 * tap + 1, tap, 1);
        kstep(I2{}, 2 * tap + 2, tap + 1, 0);
        kstep(I3{}, 2 * tap + 3, tap + 1, 1);
      }
      kstep(I0{}, 2 * (K - 1), K - 1, 0);
      kstep(I1{}, 2 * (K - 1) + 1, K - 1, 1);
    }
  };

  {
    f32x4 acc[2][NB1];
    conv(std::integral_constant<int, NB1>{}, p.w1, A_OFF, NB1 * rg, D, acc);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ch = 32 * cp + 16 * j + 4 * g;
      const float4 bb = *reinterpret_cast<const float4 *>(p.b1 + ch);
      // T row r = sample t0 - HK + r
#pragma unroll
      for (int b = 0; b < NB1; ++b) {
        const int blk = NB1 * rg + b;
        if (blk < NBT) {  // wave-uniform
          const int R = 16 * blk + r16, s = t0 - HK + R;
          // zero padding of conv2's input as a multiply (a select here became a branch per
          // element; rows that see stale LDS are never read)
          const float m = (unsigned)s < (unsigned)T ? 1.f : 0.f;
          bf16x4 t;
          t[0] = (bf16)(lrelu(acc[j][b][0] + bb.x, 0.1f) * m);
          t[1] = (bf16)(lrelu(acc[j][b][1] + bb.y, 0.1f) * m);
          t[2] = (bf16)(lrelu(acc[j][b][2] + bb.z, 0.1f) * m);
          t[3] = (bf16)(lrelu(acc[j][b][3] + bb.w, 0.1f) * m);
          *reinterpret_cast<bf16x4 *>(smem + T_OFF + R * RB + Q::phys(R, ch >> 3) * 16 + (ch & 7) * 2) = t;
        }
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
  __builtin_amdgcn_s_barrier();

  f32x4 acc[2][NB2];
  conv(std::integral_constant<int, NB2>{}, p.w2, T_OFF, NB2 * rg, 1, acc);
  // the running sum (first in the load queue after conv2's last weight wait)
  bf16x4 xs[2][NB2];
  if (p.xs != nullptr) {
    const rsrc_t sr = make_rsrc(p.xs, p.x_bytes);
#pragma unroll
    for (int b = 0; b < NB2; ++b) {
      const int s = t0 + 16 * (NB2 * rg + b) + r16;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t off = s < T ? (uint32_t)((ubase + s) * RB + (32 * cp + 16 * j + 4 * g) * 2) : kOOB;
        xs[j][b] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(sr, off, 0, 0));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
  __builtin_amdgcn_s_barrier();  // every wave done reading T: its rows 0 .. L - 1 become the output stage
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ch = 32 * cp + 16 * j + 4 * g;
    const float4 bb = *reinterpret_cast<const float4 *>(p.b2 + ch);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int b = 0; b < NB2; ++b) {
      const int R = 16 * (NB2 * rg + b) + r16;
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[j][b][i] + bv[i] + (float)res[j][b][i];
        if (p.xs != nullptr) v += (float)xs[j][b][i];
        o[i] = (bf16)(p.out_act ? lrelu(v * p.out_scale, p.out_slope) : v);
      }
      *reinterpret_cast<bf16x4 *>(smem + T_OFF + R * RB + Q::phys(R, ch >> 3) * 16 + (ch & 7) * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(kMrfLgkm0);
  __builtin_amdgcn_s_barrier();
  // whole rows, 16 bytes a lane
  const rsrc_t orr = make_rsrc(p.out, p.x_bytes);
#pragma unroll
  for (int i = 0; i < L * NCK / (64 * kPrNW); ++i) {
    const int q = i * 64 * kPrNW + tid, R = q / NCK, c = q % NCK, s = t0 + R;
    const uint4 v = *reinterpret_cast<const uint4 *>(smem + T_OFF + R * RB + Q::phys(R, c) * 16);
    if (s < T)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), orr,
                                             (uint32_t)((ubase + s) * RB + c * 16), 0, 0);
  }
}

// conv_post + tanh (hifigan/models.py:145, 159-162): y[b, t] = tanh(bias + sum_{k<7, c<32}
// w[c][k] x[b, t + k - 3, c]) over the leaky_relu'd last-stage output x bf16 [B, T, 32], y f32 [B, T].
// One output channel: as an MFMA conv (N padded to 4 on 128-row tiles) it took 816 us for the 7 M
// samples of a cfg2 batch, ~7x the time to read its 450 MB input once. Here it is a streaming
// kernel: a workgroup stages 512 + 6 rows of its utterance in LDS (80-byte pitch: the 2-row-strided
// 16-byte reads of one lane group fall in distinct bank slots), each lane computes two consecutive
// samples from 8 rows with v_dot2c_f32_bf16 (bf16 pairs, f32 accumulation: the same operand
// precision as the bf16 MFMA path) against the 112 weight pairs held in registers.
constexpr int kPostL = 512;    // output samples per workgroup (2 per lane)
constexpr int kPostPitch = 80;  // LDS bytes per staged row (64 + 16)
constexpr int kPostRows = kPostL + 6;

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void post_kernel(const bf16 *__restrict__ x, const uint32_t *__restrict__ w, float bias,
                                                   int T, float *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char sx[kPostRows * kPostPitch];
  const int b = blockIdx.y, t0 = blockIdx.x * kPostL, tid = threadIdx.x;
  const bf16 *xb = x + (int64_t)b * T * 32;
  // stage rows t0 - 3 .. t0 + 514 (4 16-byte chunks each); rows outside [0, T) are the conv's zero padding
  constexpr int kChunks = kPostRows * 4, kPer = (kChunks + 255) / 256;
  uint4 v[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = tid + i * 256, r = e >> 2, t = t0 - 3 + r;
    v[i] = make_uint4(0u, 0u, 0u, 0u);
    if (e < kChunks && t >= 0 && t < T) v[i] = *reinterpret_cast<const uint4 *>(xb + (int64_t)t * 32 + (e & 3) * 8);
  }
  uint32_t wr[7][16];  // weight pairs (tap k, channels 2j, 2j + 1)
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int j = 0; j < 16; ++j) wr[k][j] = w[k * 16 + j];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = tid + i * 256;
    if (e < kChunks) *reinterpret_cast<uint4 *>(sx + (e >> 2) * kPostPitch + (e & 3) * 16) = v[i];
  }
  __syncthreads();
  // samples s0, s0 + 1 read rows s0 .. s0 + 7 (staged row r = sample + tap)
  const int s0 = 2 * tid;
  float acc0 = 0.0f, acc1 = 0.0f;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    uint32_t h[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 q = *reinterpret_cast<const uint4 *>(sx + (s0 + r) * kPostPitch + c * 16);
      h[4 * c] = q.x;
      h[4 * c + 1] = q.y;
      h[4 * c + 2] = q.z;
      h[4 * c + 3] = q.w;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const bf16x2 hv = __builtin_bit_cast(bf16x2, h[j]);
      if (r < 7) acc0 = __builtin_amdgcn_fdot2_f32_bf16(hv, __builtin_bit_cast(bf16x2, wr[r][j]), acc0, false);
      if (r >= 1) acc1 = __builtin_amdgcn_fdot2_f32_bf16(hv, __builtin_bit_cast(bf16x2, wr[r - 1][j]), acc1, false);
    }
  }
  const int t = t0 + s0;
  float *ob = out + (int64_t)b * T;
  if (t + 1 < T) {
    *reinterpret_cast<float2 *>(ob + t) = make_float2(tanhf(acc0 + bias), tanhf(acc1 + bias));
  } else if (t < T) {
    ob[t] = tanhf(acc0 + bias);
  }
}

}  // namespace

extern "C" int fs2_hifigan_post(const void *x, const void *w, float bias, int B, int T, int C, int ks, void *out,
                                fs2_stream_t stream) {
  if (x == nullptr || w == nullptr || out == nullptr || B < 0 || T < 0) return FS2_EINVAL;
  if (C != 32 || ks != 7) return FS2_EUNSUPPORTED;
  if ((T & 1) != 0) return FS2_EUNSUPPORTED;  // float2 stores: T = frames * hop is even
  if (B == 0 || T == 0) return FS2_OK;
  const dim3 grid((unsigned)((T + kPostL - 1) / kPostL), (unsigned)B);
  hipLaunchKernelGGL(post_kernel, grid, dim3(256), 0, as_stream(stream), reinterpret_cast<const bf16 *>(x),
                     reinterpret_cast<const uint32_t *>(w), bias, T, reinterpret_cast<float *>(out));
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int64_t fs2_hifigan_mrf_weight_elems(int C) {
  return C == 32 ? mrf_woff<32>(3, 0, 0) : C == 64 ? mrf_woff<64>(3, 0, 0) : C == 128 ? mrf_woff<128>(3, 0, 0) : -1;
}

extern "C" int fs2_hifigan_mrf(const void *x, const void *x_act, const void *w, const float *bias, int B, int T, int C,
                               float out_slope, void *out, fs2_stream_t stream) {
  if (x == nullptr || x_act == nullptr || w == nullptr || bias == nullptr || out == nullptr || B < 0 || T < 0)
    return FS2_EINVAL;
  if (!(C == 32 || C == 64)) return FS2_EUNSUPPORTED;
  if (out == x || out == x_act) return FS2_EINVAL;  // other tiles re-read the input's halo rows
  if (B == 0 || T == 0) return FS2_OK;
  const int64_t bytes = (int64_t)B * T * C * 2;
  if (bytes >= (1LL << 31)) return FS2_EUNSUPPORTED;
  MrfArgs p;
  p.x = reinterpret_cast<const bf16 *>(x);
  p.a0 = reinterpret_cast<const bf16 *>(x_act);
  p.w = reinterpret_cast<const bf16 *>(w);
  p.bias = bias;
  p.out = reinterpret_cast<bf16 *>(out);
  p.T = T;
  p.ntiles = (T + kMrfL - 1) / kMrfL;
  p.slope = out_slope;
  p.x_bytes = (uint32_t)bytes;
  const dim3 grid((unsigned)p.ntiles, (unsigned)B);
  if (C == 32)
    hipLaunchKernelGGL((mrf_kernel<32, 4>), grid, dim3(256), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((mrf_kernel<64, 8>), grid, dim3(512), 0, as_stream(stream), p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_hifigan_pair(const void *x, const void *w1, const float *b1, const void *w2, const float *b2, int B,
                                int T, int C, int ks, int dilation, const void *xs, float out_scale, float out_slope,
                                int out_act, void *out, fs2_stream_t stream) {
  if (x == nullptr || w1 == nullptr || b1 == nullptr || w2 == nullptr || b2 == nullptr || out == nullptr || B < 0 || T < 0)
    return FS2_EINVAL;
  if (!(C == 128 || C == 64) || !(ks == 3 || ks == 7 || ks == 11) || dilation < 1 || dilation > 5)
    return FS2_EUNSUPPORTED;
  if (out == x) return FS2_EINVAL;  // other tiles re-read the input's halo rows
  if (B == 0 || T == 0) return FS2_OK;
  const int64_t bytes = (int64_t)B * T * C * 2;
  if (bytes >= (1LL << 31)) return FS2_EUNSUPPORTED;
  PairArgs p;
  p.x = reinterpret_cast<const bf16 *>(x);
  p.w1 = reinterpret_cast<const bf16 *>(w1);
  p.w2 = reinterpret_cast<const bf16 *>(w2);
  p.b1 = b1;
  p.b2 = b2;
  p.xs = reinterpret_cast<const bf16 *>(xs);
  p.out = reinterpret_cast<bf16 *>(out);
  p.T = T;
  p.D = dilation;
  p.out_scale = out_scale;
  p.out_slope = out_slope;
  p.out_act = out_act ? 1 : 0;
  p.x_bytes = (uint32_t)bytes;
  auto go = [&](auto CC) {
    constexpr int CV = decltype(CC)::value;
    const dim3 grid((unsigned)((T + PairCfg<CV>::L - 1) / PairCfg<CV>::L), (unsigned)B);
    if (ks == 3)
      hipLaunchKernelGGL((pair_kernel<CV, 3>), grid, dim3(64 * kPrNW), 0, as_stream(stream), p);
    else if (ks == 7)
      hipLaunchKernelGGL((pair_kernel<CV, 7>), grid, dim3(64 * kPrNW), 0, as_stream(stream), p);
    else
      hipLaunchKernelGGL((pair_kernel<CV, 11>), grid, dim3(64 * kPrNW), 0, as_stream(stream), p);
  };
  if (C == 128)
    go(std::integral_constant<int, 128>{});
  else
    go(std::integral_constant<int, 64>{});
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
