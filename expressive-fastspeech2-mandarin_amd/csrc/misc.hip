// Small bandwidth kernels around the GEMMs: encoder embedding + position encoding, the
// per-utterance speaker/emotion conditioning vectors, and the pitch/energy bucketize +
// embedding add of the VarianceAdaptor.
#include "fs2_common.h"
#include "cond.h"

namespace {

// out[b,l,:] = table[tok, :] + pe[l, :]          (transformer/Models.py:82-91)
// A token outside [0, vocab) (the reference's nn.Embedding raises IndexError / a device assert)
// makes its row NaN and increments *bad (optional device counter) -- never a silent clamp.
template <typename TO>
__global__ __launch_bounds__(256) void embed_pe_kernel(const int64_t *__restrict__ tokens, const float *__restrict__ table,
                                                       int vocab, const float *__restrict__ pe, int L, int D,
                                                       int64_t rows, TO *__restrict__ out, int32_t *__restrict__ bad) {
  const int vpr = D >> 3;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * vpr) return;
  const int64_t row = e / vpr;
  const int col = (int)(e - row * vpr) << 3;
  const int l = (int)(row % L);
  const int64_t tok = tokens[row];
  float v[8], p[8];
  if (tok < 0 || tok >= vocab) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = __builtin_nanf("");
    store8(out + row * D + col, v);
    if (bad != nullptr && col == 0) atomicAdd(bad, 1);
    return;
  }
  load8(table + tok * D + col, v);
  load8(pe + (int64_t)l * D + col, p);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] += p[q];
  store8(out + row * D + col, v);
}

__global__ __launch_bounds__(256) void cond_kernel(CondArgs a) {
  extern __shared__ float sm[];
  cond_tile(a, blockIdx.x, blockIdx.y, threadIdx.x, sm);
}

// 32 lanes per row (inside one wave, so the read of pred[m] by every lane precedes lane 0's
// write-back), 8 channels per lane per step.                   (model/modules.py:80-100)
template <typename TX>
__global__ __launch_bounds__(256) void variance_embed_kernel(const TX *x, TX *out, const float *pred, float *pred_out,
                                                             const float *__restrict__ target, float control,
                                                             const float *__restrict__ bins, int nb,
                                                             const float *__restrict__ table, int M, int D,
                                                             int64_t *__restrict__ idx_out) {
  const int m = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int sub = threadIdx.x & 31;
  if (m >= M) return;
  float v;
  if (target != nullptr) {
    v = target[m];
  } else {
    v = pred[m] * control;
  }
  // torch.bucketize(v, bins, right=False): number of boundaries strictly below v
  int lo = 0, hi = nb;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bins[mid] < v) lo = mid + 1; else hi = mid;
  }
  if (target == nullptr && pred_out != nullptr && sub == 0) pred_out[m] = v;
  if (idx_out != nullptr && sub == 0) idx_out[m] = lo;
  const float *trow = table + (int64_t)lo * D;
  const TX *xrow = x + (int64_t)m * D;
  TX *orow = out + (int64_t)m * D;
  for (int col = sub * 8; col < D; col += 256) {
    float a[8], t[8];
    load8(xrow + col, a);
    load8(trow + col, t);
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] += t[q];
    store8(orow + col, a);
  }
}

// PostNet valid-region form (runtime._postnet_valid): padded rows -> packed rows. Padded row i
// goes to packed row rowmap[i] (>= 0) of a SeqLayout; 16-byte chunks, rows of row_bytes; two
// tensors (the f32 mel and its bf16 copy) in one launch.
__global__ __launch_bounds__(256) void pack_rows_kernel(const char *__restrict__ a, int a_bytes, char *__restrict__ pa,
                                                        const char *__restrict__ b, int b_bytes, char *__restrict__ pb,
                                                        const int32_t *__restrict__ rowmap, int64_t n) {
  const int ca = a_bytes >> 4, cb = b_bytes >> 4, cpr = ca + cb;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * cpr) return;
  const int64_t i = e / cpr;
  const int c = (int)(e - i * cpr);
  const int r = rowmap[i];
  if (r < 0) return;
  if (c < ca)
    *reinterpret_cast<uint4 *>(pa + (int64_t)r * a_bytes + 16 * c) =
        *reinterpret_cast<const uint4 *>(a + i * a_bytes + 16 * c);
  else
    *reinterpret_cast<uint4 *>(pb + (int64_t)r * b_bytes + 16 * (c - ca)) =
        *reinterpret_cast<const uint4 *>(b + i * b_bytes + 16 * (c - ca));
}

// ... and back: out[b, t] = y[rowmap[b*T + t]] where exact (t < len2[b] - reach, or the whole
// utterance when len2[b] == T), else the constant row c (the PostNet of all-padding input) or,
// in the last `reach` frames before T, row t - (T - reach) of the tail block.
__global__ __launch_bounds__(256) void postnet_assemble_kernel(const float *__restrict__ y, const int32_t *__restrict__ rowmap,
                                                               const int32_t *__restrict__ cu, int T, int C,
                                                               const float *__restrict__ crow, const float *__restrict__ tail,
                                                               int reach, int64_t n, float *__restrict__ out) {
  const int v4 = C >> 2;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * v4) return;
  const int64_t i = e / v4;
  const int c = (int)(e - i * v4) * 4;
  const int bq = (int)(i / T), t = (int)(i - (int64_t)bq * T);
  const int l2 = cu[bq + 1] - cu[bq];
  const float *src;
  if (l2 >= T || t < l2 - reach)
    src = y + (int64_t)rowmap[i] * C;
  else if (t >= T - reach)
    src = tail + (int64_t)(t - (T - reach)) * C;
  else
    src = crow;
  *reinterpret_cast<float4 *>(out + i * C + c) = *reinterpret_cast<const float4 *>(src + c);
}

}  // namespace

extern "C" int fs2_embed_pe(const int64_t *tokens, const float *table, int vocab, const float *pe, int B, int L, int D,
                            void *out, int out_dtype, int32_t *bad_ids, fs2_stream_t stream) {
  if (tokens == nullptr || table == nullptr || pe == nullptr || out == nullptr) return FS2_EINVAL;
  if (B < 0 || L < 0 || D <= 0 || (D & 7) || vocab <= 0) return FS2_EINVAL;
  const int64_t rows = (int64_t)B * L;
  if (rows == 0) return FS2_OK;
  const int64_t work = rows * (D >> 3);
  dim3 grid((unsigned)((work + 255) / 256));
  hipStream_t s = as_stream(stream);
  if (out_dtype == FS2_F32)
    hipLaunchKernelGGL(embed_pe_kernel<float>, grid, dim3(256), 0, s, tokens, table, vocab, pe, L, D, rows,
                       reinterpret_cast<float *>(out), bad_ids);
  else if (out_dtype == FS2_BF16)
    hipLaunchKernelGGL(embed_pe_kernel<bf16>, grid, dim3(256), 0, s, tokens, table, vocab, pe, L, D, rows,
                       reinterpret_cast<bf16 *>(out), bad_ids);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_cond_vectors(const int64_t *speakers, const float *speaker_table, int n_speaker,
                                const int64_t *emotions, const float *emo_table, int n_emo, int d_emo,
                                const int64_t *arousals, const float *aro_table, int n_aro, int d_aro,
                                const int64_t *valences, const float *val_table, int n_val, int d_val,
                                const float *lin_w, const float *lin_b, int B, int D, float *spk_out, float *emo_out,
                                fs2_stream_t stream) {
  if (B < 0 || D <= 0) return FS2_EINVAL;
  if (speaker_table != nullptr && (speakers == nullptr || spk_out == nullptr || n_speaker <= 0)) return FS2_EINVAL;
  if (emo_table != nullptr &&
      (emotions == nullptr || arousals == nullptr || valences == nullptr || aro_table == nullptr ||
       val_table == nullptr || lin_w == nullptr || lin_b == nullptr || emo_out == nullptr || n_emo <= 0 ||
       n_aro <= 0 || n_val <= 0))
    return FS2_EINVAL;
  if (B == 0 || (speaker_table == nullptr && emo_table == nullptr)) return FS2_OK;
  const int dc = emo_table != nullptr ? d_emo + d_aro + d_val : 0;
  const size_t smem = (size_t)kCondU * (dc + 256) * sizeof(float);
  if (smem > 65536) return FS2_EUNSUPPORTED;
  CondArgs a{speakers, speaker_table, n_speaker, emotions, emo_table, n_emo, d_emo, arousals, aro_table, n_aro, d_aro,
             valences, val_table, n_val, d_val, lin_w, lin_b, B, D, spk_out, emo_out};
  hipLaunchKernelGGL(cond_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)((B + kCondU - 1) / kCondU)), dim3(256), smem,
                     as_stream(stream), a);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

static int variance_embed_launch(const void *x, int x_dtype, void *out, const float *pred, float *pred_out,
                                 const float *target, float control, const float *bins, int n_bins,
                                 const float *table, int M, int D, int64_t *idx_out, fs2_stream_t stream) {
  if (x == nullptr || out == nullptr || (pred == nullptr && target == nullptr) || bins == nullptr || table == nullptr)
    return FS2_EINVAL;
  if (M < 0 || D <= 0 || (D & 7) || n_bins < 2) return FS2_EINVAL;
  if (M == 0) return FS2_OK;
  dim3 grid((M + 7) / 8);
  hipStream_t s = as_stream(stream);
  if (x_dtype == FS2_F32)
    hipLaunchKernelGGL(variance_embed_kernel<float>, grid, dim3(256), 0, s, reinterpret_cast<const float *>(x),
                       reinterpret_cast<float *>(out), pred, pred_out, target, control, bins, n_bins - 1, table, M, D,
                       idx_out);
  else if (x_dtype == FS2_BF16)
    hipLaunchKernelGGL(variance_embed_kernel<bf16>, grid, dim3(256), 0, s, reinterpret_cast<const bf16 *>(x),
                       reinterpret_cast<bf16 *>(out), pred, pred_out, target, control, bins, n_bins - 1, table, M, D,
                       idx_out);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_variance_embed(void *x, int x_dtype, float *pred, const float *target, float control,
                                  const float *bins, int n_bins, const float *table, int M, int D,
                                  fs2_stream_t stream) {
  if (pred == nullptr) return FS2_EINVAL;
  return variance_embed_launch(x, x_dtype, x, pred, pred, target, control, bins, n_bins, table, M, D, nullptr, stream);
}

extern "C" int fs2_variance_embed_ex(const void *x, int x_dtype, const float *value, const float *bins, int n_bins,
                                     const float *table, int M, int D, void *out, int64_t *idx_out,
                                     fs2_stream_t stream) {
  if (value == nullptr) return FS2_EINVAL;
  return variance_embed_launch(x, x_dtype, out, nullptr, nullptr, value, 1.0f, bins, n_bins, table, M, D, idx_out,
                               stream);
}

extern "C" const char *fs2_version(void) { return "fs2hip 0.1.0 (gfx950)"; }

#ifndef FS2_BUILD_ID
#define FS2_BUILD_ID "unset"
#endif
extern "C" const char *fs2_build_id(void) { return FS2_BUILD_ID; }

extern "C" const char *fs2_status_string(int status) {
  switch (status) {
    case FS2_OK: return "ok";
    case FS2_EINVAL: return "invalid argument";
    case FS2_ELAUNCH: return "kernel launch failed";
    case FS2_EUNSUPPORTED: return "unsupported dtype/configuration";
    default: return "unknown status";
  }
}

extern "C" int fs2_pack_rows(const void *a, int a_row_bytes, void *packed_a, const void *b, int b_row_bytes,
                             void *packed_b, const int32_t *rowmap, int64_t n_rows, fs2_stream_t stream) {
  if (a == nullptr || packed_a == nullptr || rowmap == nullptr || n_rows < 0 || a_row_bytes <= 0 || (a_row_bytes & 15))
    return FS2_EINVAL;
  if (b != nullptr && (packed_b == nullptr || b_row_bytes <= 0 || (b_row_bytes & 15))) return FS2_EINVAL;
  if (b == nullptr) b_row_bytes = 0;
  const int64_t work = n_rows * ((a_row_bytes + b_row_bytes) >> 4);
  if (work == 0) return FS2_OK;
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const char *>(a), a_row_bytes, static_cast<char *>(packed_a),
                     static_cast<const char *>(b), b_row_bytes, static_cast<char *>(packed_b), rowmap, n_rows);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_postnet_assemble(const float *y_packed, const int32_t *rowmap, const int32_t *cu, int B, int T,
                                    int C, const float *const_row, const float *tail, int reach, float *out,
                                    fs2_stream_t stream) {
  if (y_packed == nullptr || rowmap == nullptr || cu == nullptr || const_row == nullptr || tail == nullptr ||
      out == nullptr || B < 0 || T < 0 || C <= 0 || (C & 3) || reach < 0 || reach > T)
    return FS2_EINVAL;
  const int64_t n = (int64_t)B * T, work = n * (C >> 2);
  if (work == 0) return FS2_OK;
  hipLaunchKernelGGL(postnet_assemble_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, as_stream(stream),
                     y_packed, rowmap, cu, T, C, const_row, tail, reach, n, out);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
