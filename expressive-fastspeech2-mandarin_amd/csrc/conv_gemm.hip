// Implicit-GEMM Conv1d / Linear for CDNA4 (gfx950) on MFMA, with fused epilogues.
//
//   y[b,t,n] = epi( sum_k sum_c x[b, t+k-pad, c] * w[n][k][c] + bias[n] )
//
// Every projection of the FastSpeech2 forward is this one operator (see include/fs2hip.h):
// the fused Q|K|V projection (N=768), the attention output projection + residual +
// LayerNorm + padding mask, the FFN Conv1d(k=9) + ReLU and Conv1d(k=1) + residual + LN + mask,
// the VariancePredictor Conv1d(k=3) + ReLU + LN (+ Linear(256->1) + mask), mel_linear and the
// PostNet Conv1d(k=5) (+ folded BatchNorm) + tanh / + residual.
//
// Geometry. Rows are the flattened (b, t) pairs, M = B*T; a workgroup owns a BM x BN output
// tile (4 waves, each a 64 x 64 sub-tile of 4 x 4 MFMA 16x16 blocks). The K loop runs over
// (tap, channel block) k-steps of 128 bytes per row; for tap k the A rows are the input rows
// shifted by k-pad, read with a per-row validity test (same sequence and inside [0, T)), so
// conv taps never leak across sequences and tiles may straddle sequence boundaries (no
// per-sequence tail waste). A and B tiles are staged global -> registers -> LDS, double
// buffered (loads for step k+1 are in flight while step k's MFMAs run), in 128-byte LDS rows
// whose 16-byte chunks are XOR-swizzled by (row & 7) so the ds_read_b128 fragment reads are
// bank-conflict free.
//
// Compute types: bf16 (mfma_f32_16x16x32_bf16; k-steps of 64 = 2 MFMA k-slices) or f32
// (mfma_f32_16x16x4f32, an exact f32 FMA chain; k-steps of 32). For f32 each lane reads 4
// consecutive k of its row with one ds_read_b128 and issues 4 MFMAs, MFMA j taking element j:
// A and B use the same k permutation, so the products summed are the same.
//
// Epilogue: the f32 accumulator tile goes through LDS (reusing the staging buffers) and is
// written row-major with 8/16-byte stores; the LayerNorm epilogues run one wave per row
// (N = 256 = 64 lanes x 4) with shuffle reductions.
#include "fs2_common.h"

namespace {

constexpr int kRowBytes = 128;  // one k-step of one tile row

__device__ __forceinline__ int lds_off(int row, int chunk) { return row * kRowBytes + ((chunk ^ (row & 7)) << 4); }

template <int CT>
struct CTraits;
template <>
struct CTraits<FS2_BF16> {
  static constexpr int KE = 64;  // elements per k-step
  static constexpr int CE = 8;   // elements per 16-byte chunk
  using T = bf16;
};
template <>
struct CTraits<FS2_F32> {
  static constexpr int KE = 32;
  static constexpr int CE = 4;
  using T = float;
};

// One 16-byte LDS chunk (CE compute elements) staged in registers from an input of type TIn.
template <int CT, typename TIn>
struct Stage;
template <>
struct Stage<FS2_BF16, bf16> {
  uint4 r;
  __device__ __forceinline__ void load(const bf16 *p) { r = *reinterpret_cast<const uint4 *>(p); }
  __device__ __forceinline__ void zero() { r = make_uint4(0u, 0u, 0u, 0u); }
  __device__ __forceinline__ uint4 chunk() const { return r; }
};
template <>
struct Stage<FS2_BF16, float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float *p) {
    a = reinterpret_cast<const float4 *>(p)[0];
    b = reinterpret_cast<const float4 *>(p)[1];
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ uint4 chunk() const {
    bf16x8 v = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
    return *reinterpret_cast<uint4 *>(&v);
  }
};
template <>
struct Stage<FS2_F32, float> {
  uint4 r;
  __device__ __forceinline__ void load(const float *p) { r = *reinterpret_cast<const uint4 *>(p); }
  __device__ __forceinline__ void zero() { r = make_uint4(0u, 0u, 0u, 0u); }
  __device__ __forceinline__ uint4 chunk() const { return r; }
};
template <>
struct Stage<FS2_F32, bf16> {
  uint2 r;
  __device__ __forceinline__ void load(const bf16 *p) { r = *reinterpret_cast<const uint2 *>(p); }
  __device__ __forceinline__ void zero() { r = make_uint2(0u, 0u); }
  __device__ __forceinline__ uint4 chunk() const {
    return make_uint4(r.x << 16, r.x & 0xffff0000u, r.y << 16, r.y & 0xffff0000u);
  }
};

struct ConvArgs {
  const void *x;
  int64_t xs;
  const void *w;
  const float *bias;
  int B, T, Cin, Cin_pad, N, KS, pad, M;
  int epi;
  const void *res;
  int res_dt;
  int64_t rs;
  const float *gamma;
  const float *beta;
  float eps;
  const int64_t *lens;
  const float *av1;
  const float *av2;
  const float *dw;
  float db;
  void *out;
  int out_dt;
  int64_t os;
};

__device__ __forceinline__ void load_any4(const void *p, int dt, int64_t off, float v[4]) {
  if (dt == FS2_BF16)
    load4(reinterpret_cast<const bf16 *>(p) + off, v);
  else
    load4(reinterpret_cast<const float *>(p) + off, v);
}
__device__ __forceinline__ void store_any4(void *p, int dt, int64_t off, const float v[4]) {
  if (dt == FS2_BF16)
    store4(reinterpret_cast<bf16 *>(p) + off, v);
  else
    store4(reinterpret_cast<float *>(p) + off, v);
}

template <int CT, int WGM, int WGN, typename TIn>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvArgs a) {
  constexpr int BM = 64 * WGM, BN = 64 * WGN;
  constexpr int KE = CTraits<CT>::KE, CE = CTraits<CT>::CE;
  using TW = typename CTraits<CT>::T;
  constexpr int A_CH = BM * 8 / 256, B_CH = BN * 8 / 256;
  constexpr int STAGE_BYTES = (BM + BN) * kRowBytes;
  constexpr int EPI_LD = BN + 4;
  constexpr int SMEM = (2 * STAGE_BYTES > BM * EPI_LD * 4) ? 2 * STAGE_BYTES : BM * EPI_LD * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WGN, wc = wid % WGN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int nCk = a.Cin_pad / KE;
  const int nK = a.KS * nCk;
  const int T = a.T, M = a.M;

  const TIn *__restrict__ x = reinterpret_cast<const TIn *>(a.x);
  const TW *__restrict__ w = reinterpret_cast<const TW *>(a.w);

  const int srow = tid >> 3, schunk = tid & 7;
  int a_t[A_CH];
  int a_m[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int j = 0; j < A_CH; ++j) {
    const int m = m0 + srow + 32 * j;
    a_ok[j] = m < M;
    a_m[j] = m;
    const int bb = m / T;
    a_t[j] = m - bb * T;
  }
  const TW *wp[B_CH];
  bool b_ok[B_CH];
  const int64_t wrow = (int64_t)a.KS * a.Cin_pad;
#pragma unroll
  for (int j = 0; j < B_CH; ++j) {
    const int n = n0 + srow + 32 * j;
    b_ok[j] = n < a.N;
    wp[j] = w + (int64_t)(b_ok[j] ? n : 0) * wrow + schunk * CE;
  }

  Stage<CT, TIn> sa[A_CH];
  Stage<CT, TW> sb[B_CH];

  auto gload = [&](int ks) {
    const int tap = ks / nCk;
    const int cb = ks - tap * nCk;
    const int ch = cb * KE + schunk * CE;
    const int sh = tap - a.pad;
    const bool ch_ok = ch < a.Cin;
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int ts = a_t[j] + sh;
      if (a_ok[j] && ch_ok && ts >= 0 && ts < T)
        sa[j].load(x + (int64_t)(a_m[j] + sh) * a.xs + ch);
      else
        sa[j].zero();
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      if (b_ok[j])
        sb[j].load(wp[j] + (int64_t)ks * KE);
      else
        sb[j].zero();
    }
  };
  auto lstore = [&](int buf) {
    char *As = smem + buf * STAGE_BYTES;
    char *Bs = As + BM * kRowBytes;
#pragma unroll
    for (int j = 0; j < A_CH; ++j) *reinterpret_cast<uint4 *>(As + lds_off(srow + 32 * j, schunk)) = sa[j].chunk();
#pragma unroll
    for (int j = 0; j < B_CH; ++j) *reinterpret_cast<uint4 *>(Bs + lds_off(srow + 32 * j, schunk)) = sb[j].chunk();
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nK; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nK) gload(ks + 1);
    const char *As = smem + cur * STAGE_BYTES;
    const char *Bs = As + BM * kRowBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      if constexpr (CT == FS2_BF16) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          af[mi] = *reinterpret_cast<const bf16x8 *>(As + lds_off(wr * 64 + mi * 16 + (lane & 15), ch));
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          bfr[ni] = *reinterpret_cast<const bf16x8 *>(Bs + lds_off(wc * 64 + ni * 16 + (lane & 15), ch));
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      } else {
        f32x4 af[4], bfr[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          af[mi] = *reinterpret_cast<const f32x4 *>(As + lds_off(wr * 64 + mi * 16 + (lane & 15), ch));
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          bfr[ni] = *reinterpret_cast<const f32x4 *>(Bs + lds_off(wc * 64 + ni * 16 + (lane & 15), ch));
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi][j], bfr[ni][j], acc[mi][ni], 0, 0, 0);
      }
    }
    if (ks + 1 < nK) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: accumulator tile -> LDS (f32, row-major, padded rows) -------------------------
  float *E = reinterpret_cast<float *>(smem);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        E[(wr * 64 + mi * 16 + 4 * (lane >> 4) + j) * EPI_LD + wc * 64 + ni * 16 + (lane & 15)] = acc[mi][ni][j];
  __syncthreads();

  const int epi = a.epi;
  if (epi == FS2_EPI_RES_LN || epi == FS2_EPI_RELU_LN || epi == FS2_EPI_RELU_LN_DOT) {
    // one wave per row; N == BN == 256 (checked on the host), lane owns columns 4*lane..4*lane+3
    const int n = lane * 4;
    float bias4[4], g4[4], be4[4];
    load4(a.gamma + n, g4);
    load4(a.beta + n, be4);
#pragma unroll
    for (int q = 0; q < 4; ++q) bias4[q] = a.bias[n + q];
    const float inv_n = 1.0f / (float)a.N;
    for (int r = wid; r < BM; r += 4) {
      const int m = m0 + r;
      if (m >= M) break;
      float v[4];
      load4(E + r * EPI_LD + n, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += bias4[q];
      if (epi == FS2_EPI_RES_LN) {
        float rv[4];
        load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += rv[q];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.0f);
      }
      const float mean = wave_sum(v[0] + v[1] + v[2] + v[3]) * inv_n;
      float d[4], ss = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[q] = v[q] - mean;
        ss += d[q] * d[q];
      }
      const float var = wave_sum(ss) * inv_n;
      const float rstd = 1.0f / sqrtf(var + a.eps);
      float y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = d[q] * rstd * g4[q] + be4[q];
      const int bb = m / T;
      const int t = m - bb * T;
      const bool masked = (a.lens != nullptr) && ((int64_t)t >= a.lens[bb]);
      if (epi == FS2_EPI_RELU_LN_DOT) {
        float dw4[4];
        load4(a.dw + n, dw4);
        const float s = wave_sum(y[0] * dw4[0] + y[1] * dw4[1] + y[2] * dw4[2] + y[3] * dw4[3]) + a.db;
        if (lane == 0) reinterpret_cast<float *>(a.out)[m] = masked ? 0.0f : s;
        continue;
      }
      if (epi == FS2_EPI_RES_LN) {
        if (masked) {
#pragma unroll
          for (int q = 0; q < 4; ++q) y[q] = 0.0f;
        }
        if (a.av1 != nullptr) {
          float av[4];
          load4(a.av1 + (int64_t)bb * a.N + n, av);
#pragma unroll
          for (int q = 0; q < 4; ++q) y[q] += av[q];
        }
        if (a.av2 != nullptr) {
          float av[4];
          load4(a.av2 + (int64_t)bb * a.N + n, av);
#pragma unroll
          for (int q = 0; q < 4; ++q) y[q] += av[q];
        }
      }
      store_any4(a.out, a.out_dt, (int64_t)m * a.os + n, y);
    }
    return;
  }

  constexpr int G = BN / 4;
  for (int e = tid; e < BM * G; e += 256) {
    const int r = e / G;
    const int cg = e - r * G;
    const int m = m0 + r;
    const int n = n0 + cg * 4;
    if (m >= M || n >= a.N) continue;
    float v[4];
    load4(E + r * EPI_LD + cg * 4, v);
    if (a.bias != nullptr) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += a.bias[n + q];
    }
    if (epi == FS2_EPI_BIAS_RELU) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.0f);
    } else if (epi == FS2_EPI_BIAS_TANH) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
    } else if (epi == FS2_EPI_BIAS_RES) {
      float rv[4];
      load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += rv[q];
    }
    store_any4(a.out, a.out_dt, (int64_t)m * a.os + n, v);
  }
}

template <int CT, int WGM, int WGN, typename TIn>
void launch(const ConvArgs &a, hipStream_t s) {
  constexpr int BM = 64 * WGM, BN = 64 * WGN;
  dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN);
  hipLaunchKernelGGL((conv_gemm_kernel<CT, WGM, WGN, TIn>), grid, dim3(256), 0, s, a);
}

}  // namespace

extern "C" int fs2_conv_cin_pad(int Cin, int compute) {
  const int ke = compute == FS2_BF16 ? CTraits<FS2_BF16>::KE : CTraits<FS2_F32>::KE;
  return (Cin + ke - 1) / ke * ke;
}

extern "C" int fs2_conv1d(const fs2_conv_desc *d, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->out == nullptr) return FS2_EINVAL;
  if (d->compute != FS2_BF16 && d->compute != FS2_F32) return FS2_EUNSUPPORTED;
  const int ce = d->compute == FS2_BF16 ? 8 : 4;
  if (d->B < 0 || d->T < 0 || d->Cin <= 0 || d->N <= 0 || d->KS <= 0 || d->pad < 0) return FS2_EINVAL;
  if (d->Cin % ce != 0 || d->N % 4 != 0 || d->Cin_pad != fs2_conv_cin_pad(d->Cin, d->compute)) return FS2_EINVAL;
  if (d->x_row_stride < d->Cin || (d->x_row_stride % ce) != 0) return FS2_EINVAL;
  const int epi = d->epilogue;
  if (epi < FS2_EPI_BIAS || epi > FS2_EPI_RELU_LN_DOT) return FS2_EINVAL;
  const bool ln = epi == FS2_EPI_RES_LN || epi == FS2_EPI_RELU_LN || epi == FS2_EPI_RELU_LN_DOT;
  if (ln && (d->N != 256 || d->ln_gamma == nullptr || d->ln_beta == nullptr || d->bias == nullptr)) return FS2_EINVAL;
  if ((epi == FS2_EPI_RES_LN || epi == FS2_EPI_BIAS_RES) && d->residual == nullptr) return FS2_EINVAL;
  if (epi == FS2_EPI_RELU_LN_DOT && (d->dot_w == nullptr || d->out_dtype != FS2_F32)) return FS2_EINVAL;
  if (epi != FS2_EPI_RELU_LN_DOT && (d->out_row_stride < d->N || (d->out_row_stride & 3) != 0)) return FS2_EINVAL;
  if ((epi == FS2_EPI_RES_LN || epi == FS2_EPI_BIAS_RES) && (d->res_row_stride < d->N || (d->res_row_stride & 3)))
    return FS2_EINVAL;
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 > 0x7fffff00LL) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;

  ConvArgs a;
  a.x = d->x;
  a.xs = d->x_row_stride;
  a.w = d->w;
  a.bias = d->bias;
  a.B = d->B;
  a.T = d->T;
  a.Cin = d->Cin;
  a.Cin_pad = d->Cin_pad;
  a.N = d->N;
  a.KS = d->KS;
  a.pad = d->pad;
  a.M = (int)M64;
  a.epi = epi;
  a.res = d->residual;
  a.res_dt = d->res_dtype;
  a.rs = d->res_row_stride;
  a.gamma = d->ln_gamma;
  a.beta = d->ln_beta;
  a.eps = d->ln_eps;
  a.lens = d->lens;
  a.av1 = d->addvec1;
  a.av2 = d->addvec2;
  a.dw = d->dot_w;
  a.db = d->dot_b;
  a.out = d->out;
  a.out_dt = d->out_dtype;
  a.os = d->out_row_stride;

  hipStream_t s = as_stream(stream);
  const bool xb = d->x_dtype == FS2_BF16;
  if (d->x_dtype != FS2_BF16 && d->x_dtype != FS2_F32) return FS2_EUNSUPPORTED;
  if (d->compute == FS2_BF16) {
    if (ln)
      xb ? launch<FS2_BF16, 1, 4, bf16>(a, s) : launch<FS2_BF16, 1, 4, float>(a, s);
    else
      xb ? launch<FS2_BF16, 2, 2, bf16>(a, s) : launch<FS2_BF16, 2, 2, float>(a, s);
  } else {
    if (ln)
      xb ? launch<FS2_F32, 1, 4, bf16>(a, s) : launch<FS2_F32, 1, 4, float>(a, s);
    else
      xb ? launch<FS2_F32, 2, 2, bf16>(a, s) : launch<FS2_F32, 2, 2, float>(a, s);
  }
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
