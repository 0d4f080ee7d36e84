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

}  // namespace

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
