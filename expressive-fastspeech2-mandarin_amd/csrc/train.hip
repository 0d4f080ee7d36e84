// Training-step kernels around the GEMMs (train.py step, cfg3): the FFT block's
//   y = masked_fill(LayerNorm(dropout(a) + res), pad, 0)            (transformer/SubLayers.py:54-57,90-93,
//                                                                      transformer/Layers.py:27-30)
// forward in one pass per row, its backward (input, residual, gamma/beta and the producing
// conv's bias gradients) in one pass plus a deterministic column reduction, and a generic
// deterministic column sum (bias gradients of the other convs).
//
// Dropout keep bits come from a counter hash of (seed, salt, row, column): the backward
// regenerates them instead of storing a mask. The seed lives in device memory (one int64 that the
// trainer advances once per step inside the captured graph), so graph replays draw fresh masks.
#include "fs2_common.h"

namespace {

constexpr int kD = 256;       // d_model (transformer.encoder_hidden / decoder_hidden)
constexpr int kLnBlocks = 256; // partial-sum blocks of the LN backward

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_key(const int64_t *seed, uint32_t salt) {
  const uint64_t s = seed != nullptr ? (uint64_t)*seed : 0ull;
  return mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + salt * 0x9E3779B9U));
}

// keep mask of 4 consecutive columns as 4 bits
__device__ __forceinline__ unsigned keep4(uint32_t key, uint32_t idx0, uint32_t thr) {
  unsigned m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) m |= ((mix32((idx0 + q) ^ key) >> 8) >= thr ? 1u : 0u) << q;
  return m;
}

__device__ __forceinline__ bool row_masked(const int64_t *lens, int64_t row, int T) {
  if (lens == nullptr) return false;
  const int64_t b = row / T;
  return row - b * T >= lens[b];
}

// Deterministic split-partial sums for the finish kernels: a 256-thread block = 4 row groups x 64
// columns; row group g sums partials g, g+4, ... (two independent accumulators, unrolled loads),
// the 4 group sums are added in a fixed order through LDS. Every thread of the block must call it
// (it synchronises); the result is valid in all threads of the column.
__device__ __forceinline__ float parts_col_sum(const float *__restrict__ part, int S, int64_t M, int64_t col) {
  __shared__ float red[4][64];
  const int rg = threadIdx.x >> 6, cl = threadIdx.x & 63;
  float a0 = 0.f, a1 = 0.f;
  if (col < M) {
    int k = rg;
#pragma unroll 4
    for (; k + 4 < S; k += 8) {
      a0 += part[(int64_t)k * M + col];
      a1 += part[(int64_t)(k + 4) * M + col];
    }
    if (k < S) a0 += part[(int64_t)k * M + col];
  }
  red[rg][cl] = a0 + a1;
  __syncthreads();
  const float r = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
  __syncthreads();
  return r;
}

template <typename TR>
__global__ __launch_bounds__(256) void res_ln_fwd_kernel(const float *__restrict__ a, const TR *__restrict__ res,
                                                         const float *__restrict__ gamma, const float *__restrict__ beta,
                                                         const int64_t *__restrict__ lens, int64_t R, int T, float eps,
                                                         uint32_t thr, float scale, const int64_t *seed, uint32_t salt,
                                                         float *__restrict__ y, bf16 *__restrict__ y_bf,
                                                         float *__restrict__ xhat, float *__restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int c = lane * 4;
  const uint32_t key = drop_key(seed, salt);
  float g[4], bt[4];
  load4(gamma + c, g);
  load4(beta + c, bt);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < R; row += nw) {
    float v[4], r[4];
    load4(a + row * kD + c, v);
    load4(res + row * kD + c, r);
    if (thr != 0) {
      const unsigned k = keep4(key, (uint32_t)(row * kD + c), thr);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ((k >> q) & 1) ? v[q] * scale : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += r[q];
    const float mean = wave_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / kD);
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] -= mean;
      s2 += v[q] * v[q];
    }
    const float rs = rsqrtf(wave_sum(s2) * (1.0f / kD) + eps);
    const bool masked = row_masked(lens, row, T);
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] *= rs;
      o[q] = masked ? 0.0f : v[q] * g[q] + bt[q];
    }
    store4(xhat + row * kD + c, v);
    store4(y + row * kD + c, o);
    if (y_bf != nullptr) store4(y_bf + row * kD + c, o);
    if (lane == 0) rstd_out[row] = rs;
  }
}

// dv = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)); dres = dv; da = dv * keep * scale.
// part[blk][0..3][kD]: sum dy*xhat (gamma), sum dy (beta), sum da (the producing conv's bias).
__global__ __launch_bounds__(256) void res_ln_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ xhat,
                                                         const float *__restrict__ rstd, const float *__restrict__ gamma,
                                                         const int64_t *__restrict__ lens, int64_t R, int T, uint32_t thr,
                                                         float scale, const int64_t *seed, uint32_t salt,
                                                         float *__restrict__ dres, bf16 *__restrict__ da,
                                                         float *__restrict__ part) {
  __shared__ float red[3][4][kD];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane * 4;
  const uint32_t key = drop_key(seed, salt);
  float g[4];
  load4(gamma + c, g);
  float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f}, pa[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < R; row += nw) {
    if (row_masked(lens, row, T)) {  // masked_fill's gradient: nothing flows through a padding row
      const float z[4] = {0.f, 0.f, 0.f, 0.f};
      store4(dres + row * kD + c, z);
      store4(da + row * kD + c, z);
      continue;
    }
    float d[4], xh[4], gd[4];
    load4(dy + row * kD + c, d);
    load4(xhat + row * kD + c, xh);
    const float rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      gd[q] = g[q] * d[q];
      s1 += gd[q];
      s2 += gd[q] * xh[q];
      pg[q] += d[q] * xh[q];
      pb[q] += d[q];
    }
    const float m1 = wave_sum(s1) * (1.0f / kD), m2 = wave_sum(s2) * (1.0f / kD);
    float dv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dv[q] = rs * (gd[q] - m1 - xh[q] * m2);
    store4(dres + row * kD + c, dv);
    if (thr != 0) {
      const unsigned k = keep4(key, (uint32_t)(row * kD + c), thr);
#pragma unroll
      for (int q = 0; q < 4; ++q) dv[q] = ((k >> q) & 1) ? dv[q] * scale : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) pa[q] += dv[q];
    store4(da + row * kD + c, dv);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[0][wv][c + q] = pg[q];
    red[1][wv][c + q] = pb[q];
    red[2][wv][c + q] = pa[q];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * kD; i += 256) {
    const int k = i / kD, col = i - k * kD;
    part[(int64_t)blockIdx.x * 3 * kD + i] = (red[k][0][col] + red[k][1][col]) + (red[k][2][col] + red[k][3][col]);
  }
}

// VariancePredictor layer (model/modules.py:218-235, train mode): y = dropout(LN(relu(a))).
// Saves xhat / rstd; the backward reads a again for the relu mask. HEAD (the predictor's second
// layer): also the predictor's output, out[r] = masked ? 0 : y[r] . hw + hb (linear_layer + squeeze
// + masked_fill, modules.py:245-250) from the row still in registers; y itself is then not stored
// (nothing else reads it).
template <bool HEAD>
__global__ __launch_bounds__(256) void relu_ln_fwd_kernel(const float *__restrict__ a, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta, int64_t R, float eps,
                                                          uint32_t thr, float scale, const int64_t *seed, uint32_t salt,
                                                          float *__restrict__ y, bf16 *__restrict__ y_bf,
                                                          float *__restrict__ xhat, float *__restrict__ rstd_out,
                                                          const float *__restrict__ hw, const float *__restrict__ hb,
                                                          const bool *__restrict__ hmask, float *__restrict__ hout) {
  const int lane = threadIdx.x & 63;
  const int c = lane * 4;
  const uint32_t key = drop_key(seed, salt);
  float g[4], bt[4], w4[4] = {0.f, 0.f, 0.f, 0.f};
  load4(gamma + c, g);
  load4(beta + c, bt);
  if constexpr (HEAD) load4(hw + c, w4);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < R; row += nw) {
    float v[4];
    load4(a + row * kD + c, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.0f);
    const float mean = wave_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / kD);
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] -= mean;
      s2 += v[q] * v[q];
    }
    const float rs = rsqrtf(wave_sum(s2) * (1.0f / kD) + eps);
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] *= rs;
      o[q] = v[q] * g[q] + bt[q];
    }
    if (thr != 0) {
      const unsigned k = keep4(key, (uint32_t)(row * kD + c), thr);
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = ((k >> q) & 1) ? o[q] * scale : 0.0f;
    }
    store4(xhat + row * kD + c, v);
    if (y != nullptr) store4(y + row * kD + c, o);
    if (y_bf != nullptr) store4(y_bf + row * kD + c, o);
    if constexpr (HEAD) {
      const float hs = wave_sum((o[0] * w4[0] + o[1] * w4[1]) + (o[2] * w4[2] + o[3] * w4[3]));
      if (lane == 0) hout[row] = (hmask != nullptr && hmask[row]) ? 0.0f : hs + hb[0];
    }
    if (lane == 0) rstd_out[row] = rs;
  }
}

// dz = dy * keep * scale; dr = rstd * (g*dz - mean(g*dz) - xhat * mean(g*dz*xhat)); da = dr * (a > 0)
// (bf16). part[blk][0..3][kD]: sum dz*xhat (gamma), sum dz (beta), sum da (the conv's bias).
// HEAD: dy is not read but formed from the predictor output's gradient, dy[r][c] = dm[r] * hw[c]
// (dm = masked ? 0 : dout[r]), and hpart[blk][kD + 4] gets the head's gradients: sum dm * y (its
// weight; y recomputed from xhat, gamma, beta and the dropout mask) and sum dm (its bias, col kD).
template <bool HEAD>
__global__ __launch_bounds__(256) void relu_ln_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ a,
                                                          const float *__restrict__ xhat, const float *__restrict__ rstd,
                                                          const float *__restrict__ gamma, int64_t R, uint32_t thr,
                                                          float scale, const int64_t *seed, uint32_t salt,
                                                          bf16 *__restrict__ da, float *__restrict__ part,
                                                          const float *__restrict__ dout, const bool *__restrict__ hmask,
                                                          const float *__restrict__ hw, const float *__restrict__ beta,
                                                          float *__restrict__ hpart) {
  __shared__ float red[3][4][kD];
  __shared__ float hred[HEAD ? 4 : 1][HEAD ? kD + 4 : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane * 4;
  const uint32_t key = drop_key(seed, salt);
  float g[4], w4[4] = {0.f, 0.f, 0.f, 0.f}, bt[4] = {0.f, 0.f, 0.f, 0.f};
  load4(gamma + c, g);
  if constexpr (HEAD) {
    load4(hw + c, w4);
    load4(beta + c, bt);
  }
  float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f}, pa[4] = {0.f, 0.f, 0.f, 0.f};
  float ph[4] = {0.f, 0.f, 0.f, 0.f}, phb = 0.f;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < R; row += nw) {
    float d[4], xh[4], av[4], gd[4];
    load4(xhat + row * kD + c, xh);
    load4(a + row * kD + c, av);
    unsigned keep = 0xf;
    if (thr != 0) keep = keep4(key, (uint32_t)(row * kD + c), thr);
    if constexpr (HEAD) {
      const float dm = (hmask != nullptr && hmask[row]) ? 0.0f : dout[row];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[q] = dm * w4[q];
        const float yq = ((keep >> q) & 1) ? (xh[q] * g[q] + bt[q]) * (thr != 0 ? scale : 1.0f) : 0.0f;
        ph[q] += dm * yq;
      }
      phb += dm;
    } else {
      load4(dy + row * kD + c, d);
    }
    if (thr != 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = ((keep >> q) & 1) ? d[q] * scale : 0.0f;
    }
    const float rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      gd[q] = g[q] * d[q];
      s1 += gd[q];
      s2 += gd[q] * xh[q];
      pg[q] += d[q] * xh[q];
      pb[q] += d[q];
    }
    const float m1 = wave_sum(s1) * (1.0f / kD), m2 = wave_sum(s2) * (1.0f / kD);
    float dr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dr[q] = av[q] > 0.0f ? rs * (gd[q] - m1 - xh[q] * m2) : 0.0f;
      pa[q] += dr[q];
    }
    store4(da + row * kD + c, dr);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[0][wv][c + q] = pg[q];
    red[1][wv][c + q] = pb[q];
    red[2][wv][c + q] = pa[q];
    if constexpr (HEAD) hred[wv][c + q] = ph[q];
  }
  if constexpr (HEAD) {
    if (lane < 4) hred[wv][kD + lane] = lane == 0 ? phb : 0.0f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * kD; i += 256) {
    const int k = i / kD, col = i - k * kD;
    part[(int64_t)blockIdx.x * 3 * kD + i] = (red[k][0][col] + red[k][1][col]) + (red[k][2][col] + red[k][3][col]);
  }
  if constexpr (HEAD) {
    for (int i = threadIdx.x; i < kD + 4; i += 256)
      hpart[(int64_t)blockIdx.x * (kD + 4) + i] = (hred[0][i] + hred[1][i]) + (hred[2][i] + hred[3][i]);
  }
}

// Embedding backward (nn.Embedding autograd; src_word_emb with padding_idx, pitch / energy
// bucket embeddings, speaker / emotion tables): workgroup v sums the dy rows of every position i
// with tokens[i] == v (chunks of 256 positions compacted in order through LDS) in a fixed order,
// so the result is deterministic (no atomics). Row padding_idx gets no gradient.
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t *__restrict__ tokens, int64_t n,
                                                        const float *__restrict__ dy, int64_t dys, int D,
                                                        int padding_idx, float *__restrict__ out, int accumulate) {
  __shared__ int list[256];
  __shared__ int wcnt[4];
  const int v = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float acc = 0.f;
  float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool vec = (D & 3) == 0 && (dys & 3) == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  const bool skip = v == padding_idx;
  if (!skip)
    for (int64_t base = 0; base < n; base += 256) {
      const int64_t i = base + tid;
      const bool hit = i < n && tokens[i] == (int64_t)v;
      const uint64_t m = __ballot(hit);
      if (lane == 0) wcnt[wv] = __popcll(m);
      __syncthreads();
      int off = 0;
      for (int w = 0; w < wv; ++w) off += wcnt[w];
      const int total = (wcnt[0] + wcnt[1]) + (wcnt[2] + wcnt[3]);
      if (hit) list[off + __popcll(m & ((1ull << lane) - 1ull))] = tid;
      __syncthreads();
      if (vec) {
        // D % 4 == 0: wave wv sums the chunk's hits [wv q, wv q + q) in order, a lane 4 columns
        // (16-byte loads), 8 hit rows' loads in flight before their adds; the 4 wave sums are
        // added in wave order at the end (a common pitch / energy bucket has hundreds of hits: one
        // wave's serial adds were the launch's critical path)
        const int q = (total + 3) >> 2, j0 = wv * q, j1 = j0 + q < total ? j0 + q : total;
        if (4 * lane < D) {
          int j = j0;
          for (; j + 8 <= j1; j += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4 *>(dy + (base + list[j + u]) * dys + 4 * lane);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc4.x += v[u].x, acc4.y += v[u].y, acc4.z += v[u].z, acc4.w += v[u].w;
          }
          for (; j < j1; ++j) {
            const float4 v = *reinterpret_cast<const float4 *>(dy + (base + list[j]) * dys + 4 * lane);
            acc4.x += v.x, acc4.y += v.y, acc4.z += v.z, acc4.w += v.w;
          }
        }
      } else if (tid < D) {
        // 8 hit rows' loads in flight before their adds (in order)
        int j = 0;
        for (; j + 8 <= total; j += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = dy[(base + list[j + u]) * dys + tid];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; j < total; ++j) acc += dy[(base + list[j]) * dys + tid];
      }
      __syncthreads();
    }
  if (vec) {
    __shared__ float4 red[4][64];
    red[wv][lane] = acc4;
    __syncthreads();
    if (tid < D) {
      const float *r = reinterpret_cast<const float *>(&red[0][0]);
      acc = ((r[tid] + r[256 + tid]) + r[512 + tid]) + r[768 + tid];
    }
  }
  if (tid < D) {
    float *o = out + (int64_t)v * D + tid;
    *o = accumulate ? *o + acc : acc;
  }
}

// Column sums, pass 1: block (256-column stripe, row chunk) -> part[chunk][N]; 4 columns per
// thread, 4 rows in flight per block (one per wave).
template <typename T>
__global__ __launch_bounds__(256) void colsum_part_kernel(const T *__restrict__ x, int64_t R, int N, int64_t rs,
                                                          int rows_per_chunk, float *__restrict__ part) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < R ? r0 + rows_per_chunk : R;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N)
    for (int64_t r = r0 + wv; r < r1; r += 4) {
      float v[4];
      load4(x + r * rs + c, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) s[q] += v[q];
    }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[wv][lane * 4 + q] = s[q];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < N)
    part[(int64_t)blockIdx.y * N + col] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// pass 2: out[n] (+)= sum over chunks of part[chunk][n] (parts_col_sum: deterministic)
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float *__restrict__ part, int chunks, int N,
                                                            float *__restrict__ out, int accumulate) {
  const int64_t n = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const float s = parts_col_sum(part, chunks, N, n);
  if (threadIdx.x < 64 && n < N) out[n] = accumulate ? out[n] + s : s;
}

// LN backward pass 2: (dgamma, dbeta, dbias)[n] (+)= sum over the partial blocks (part[blk][3][kD])
__global__ __launch_bounds__(256) void ln_finish_kernel(const float *__restrict__ part, int chunks, float *dgamma,
                                                        float *dbeta, float *dbias, int accumulate) {
  const int64_t col = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);  // which * kD + n
  const float s = parts_col_sum(part, chunks, 3 * kD, col);
  const int which = (int)(col / kD), n = (int)(col - (int64_t)which * kD);
  float *out = which == 0 ? dgamma : (which == 1 ? dbeta : dbias);
  if (threadIdx.x < 64 && out != nullptr) out[n] = accumulate ? out[n] + s : s;
}

uint32_t drop_threshold(float p) {
  if (!(p > 0.0f)) return 0u;
  const double t = (double)p * 16777216.0;
  return t >= 16777216.0 ? 16777216u : (uint32_t)t;
}

}  // namespace

extern "C" int fs2_res_ln_fwd(const float *a, const void *res, int res_dtype, const float *gamma, const float *beta,
                              const int64_t *lens, int64_t R, int T, int D, float eps, float p_drop,
                              const int64_t *seed, int salt, float *y, void *y_bf, float *xhat, float *rstd,
                              fs2_stream_t stream) {
  if (a == nullptr || res == nullptr || gamma == nullptr || beta == nullptr || y == nullptr || xhat == nullptr ||
      rstd == nullptr)
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R < 0 || T <= 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (lens != nullptr && R % T) return FS2_EINVAL;
  if (R == 0) return FS2_OK;
  const uint32_t thr = drop_threshold(p_drop);
  const float scale = 1.0f / (1.0f - p_drop);
  const int64_t blocks64 = (R + 3) / 4;
  const unsigned grid = (unsigned)(blocks64 < 2048 ? blocks64 : 2048);
  hipStream_t s = as_stream(stream);
  if (res_dtype == FS2_F32)
    hipLaunchKernelGGL(res_ln_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, a, reinterpret_cast<const float *>(res),
                       gamma, beta, lens, R, T, eps, thr, scale, seed, (uint32_t)salt, y,
                       reinterpret_cast<bf16 *>(y_bf), xhat, rstd);
  else if (res_dtype == FS2_BF16)
    hipLaunchKernelGGL(res_ln_fwd_kernel<bf16>, dim3(grid), dim3(256), 0, s, a, reinterpret_cast<const bf16 *>(res),
                       gamma, beta, lens, R, T, eps, thr, scale, seed, (uint32_t)salt, y,
                       reinterpret_cast<bf16 *>(y_bf), xhat, rstd);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int64_t fs2_res_ln_bwd_ws_bytes(int D) { return (int64_t)kLnBlocks * 3 * D * (int64_t)sizeof(float); }

extern "C" int fs2_res_ln_bwd(const float *dy, const float *xhat, const float *rstd, const float *gamma,
                              const int64_t *lens, int64_t R, int T, int D, float p_drop, const int64_t *seed, int salt,
                              float *dres, void *da, float *dgamma, float *dbeta, float *dbias, int accumulate,
                              int defer, float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dy == nullptr || xhat == nullptr || rstd == nullptr || gamma == nullptr || dres == nullptr || da == nullptr ||
      ((dgamma == nullptr || dbeta == nullptr) && !defer) || ws == nullptr)
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R < 0 || T <= 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (lens != nullptr && R % T) return FS2_EINVAL;
  if (ws_bytes < fs2_res_ln_bwd_ws_bytes(D)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  if (R == 0) {
    if (defer) {
      (void)hipMemsetAsync(ws, 0, 3 * kD * sizeof(float), s);  // one zero partial block
      return FS2_OK;
    }
    if (!accumulate) {
      (void)hipMemsetAsync(dgamma, 0, kD * sizeof(float), s);
      (void)hipMemsetAsync(dbeta, 0, kD * sizeof(float), s);
      if (dbias != nullptr) (void)hipMemsetAsync(dbias, 0, kD * sizeof(float), s);
    }
    return FS2_OK;
  }
  const uint32_t thr = drop_threshold(p_drop);
  const float scale = 1.0f / (1.0f - p_drop);
  const int64_t b64 = (R + 3) / 4;
  const int grid = (int)(b64 < kLnBlocks ? b64 : kLnBlocks);
  hipLaunchKernelGGL(res_ln_bwd_kernel, dim3(grid), dim3(256), 0, s, dy, xhat, rstd, gamma, lens, R, T, thr, scale,
                     seed, (uint32_t)salt, dres, reinterpret_cast<bf16 *>(da), ws);
  if (defer) {
    FS2_CHECK_LAUNCH();
    return FS2_OK;
  }
  hipLaunchKernelGGL(ln_finish_kernel, dim3(3 * kD / 64), dim3(256), 0, s, ws, grid, dgamma, dbeta, dbias, accumulate);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_relu_ln_fwd(const float *a, const float *gamma, const float *beta, int64_t R, int D, float eps,
                               float p_drop, const int64_t *seed, int salt, float *y, void *y_bf, float *xhat,
                               float *rstd, fs2_stream_t stream) {
  if (a == nullptr || gamma == nullptr || beta == nullptr || y == nullptr || xhat == nullptr || rstd == nullptr)
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R < 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (R == 0) return FS2_OK;
  const int64_t b64 = (R + 3) / 4;
  hipLaunchKernelGGL(relu_ln_fwd_kernel<false>, dim3((unsigned)(b64 < 2048 ? b64 : 2048)), dim3(256), 0,
                     as_stream(stream), a, gamma, beta, R, eps, drop_threshold(p_drop), 1.0f / (1.0f - p_drop), seed,
                     (uint32_t)salt, y, reinterpret_cast<bf16 *>(y_bf), xhat, rstd, nullptr, nullptr, nullptr, nullptr);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_relu_ln_bwd(const float *dy, const float *a, const float *xhat, const float *rstd,
                               const float *gamma, int64_t R, int D, float p_drop, const int64_t *seed, int salt,
                               void *da, float *dgamma, float *dbeta, float *dbias, int accumulate, int defer,
                               float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dy == nullptr || a == nullptr || xhat == nullptr || rstd == nullptr || gamma == nullptr || da == nullptr ||
      ((dgamma == nullptr || dbeta == nullptr) && !defer) || ws == nullptr)
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R < 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (ws_bytes < fs2_res_ln_bwd_ws_bytes(D)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  if (R == 0) {
    if (defer) {
      (void)hipMemsetAsync(ws, 0, 3 * kD * sizeof(float), s);  // one zero partial block
      return FS2_OK;
    }
    if (!accumulate) {
      (void)hipMemsetAsync(dgamma, 0, kD * sizeof(float), s);
      (void)hipMemsetAsync(dbeta, 0, kD * sizeof(float), s);
      if (dbias != nullptr) (void)hipMemsetAsync(dbias, 0, kD * sizeof(float), s);
    }
    return FS2_OK;
  }
  const int64_t b64 = (R + 3) / 4;
  const int grid = (int)(b64 < kLnBlocks ? b64 : kLnBlocks);
  hipLaunchKernelGGL(relu_ln_bwd_kernel<false>, dim3(grid), dim3(256), 0, s, dy, a, xhat, rstd, gamma, R,
                     drop_threshold(p_drop), 1.0f / (1.0f - p_drop), seed, (uint32_t)salt,
                     reinterpret_cast<bf16 *>(da), ws, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (defer) {
    FS2_CHECK_LAUNCH();
    return FS2_OK;
  }
  hipLaunchKernelGGL(ln_finish_kernel, dim3(3 * kD / 64), dim3(256), 0, s, ws, grid, dgamma, dbeta, dbias, accumulate);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// The VariancePredictor's second layer with its head (model/modules.py:230-250 in train mode): the
// relu + LN + dropout of fs2_relu_ln_fwd and out = masked_fill(y . hw + hb, mask, 0) in one launch
// (no y tensor); the backward takes dout (the predictor output's gradient) instead of dy. The head's
// gradients (dhw [kD], dhb [1]) are per-block partials in the workspace after the LN ones, finished
// here or (defer) by fs2_reduce_batch_launch kind 2.
extern "C" int64_t fs2_relu_ln_head_bwd_ws_bytes(int D) {
  return fs2_res_ln_bwd_ws_bytes(D) + (int64_t)kLnBlocks * (D + 4) * (int64_t)sizeof(float);
}

extern "C" int fs2_relu_ln_head_fwd(const float *a, const float *gamma, const float *beta, int64_t R, int D, float eps,
                                    float p_drop, const int64_t *seed, int salt, void *y_bf, float *xhat, float *rstd,
                                    const float *hw, const float *hb, const bool *hmask, float *hout,
                                    fs2_stream_t stream) {
  if (a == nullptr || gamma == nullptr || beta == nullptr || xhat == nullptr || rstd == nullptr || hw == nullptr ||
      hb == nullptr || hout == nullptr)
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R < 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (R == 0) return FS2_OK;
  const int64_t b64 = (R + 3) / 4;
  hipLaunchKernelGGL(relu_ln_fwd_kernel<true>, dim3((unsigned)(b64 < 2048 ? b64 : 2048)), dim3(256), 0,
                     as_stream(stream), a, gamma, beta, R, eps, drop_threshold(p_drop), 1.0f / (1.0f - p_drop), seed,
                     (uint32_t)salt, nullptr, reinterpret_cast<bf16 *>(y_bf), xhat, rstd, hw, hb, hmask, hout);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_relu_ln_head_bwd(const float *dout, const bool *hmask, const float *hw, const float *beta,
                                    const float *a, const float *xhat, const float *rstd, const float *gamma,
                                    int64_t R, int D, float p_drop, const int64_t *seed, int salt, void *da,
                                    float *dgamma, float *dbeta, float *dbias, float *dhw, float *dhb, int accumulate,
                                    int defer, float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dout == nullptr || hw == nullptr || beta == nullptr || a == nullptr || xhat == nullptr || rstd == nullptr ||
      gamma == nullptr || da == nullptr || ws == nullptr ||
      ((dgamma == nullptr || dbeta == nullptr || dhw == nullptr || dhb == nullptr) && !defer))
    return FS2_EINVAL;
  if (D != kD) return FS2_EUNSUPPORTED;
  if (R <= 0 || !(p_drop >= 0.0f && p_drop < 1.0f) || (p_drop > 0.0f && seed == nullptr)) return FS2_EINVAL;
  if (ws_bytes < fs2_relu_ln_head_bwd_ws_bytes(D)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  const int64_t b64 = (R + 3) / 4;
  const int grid = (int)(b64 < kLnBlocks ? b64 : kLnBlocks);
  float *hpart = ws + (int64_t)kLnBlocks * 3 * kD;
  hipLaunchKernelGGL(relu_ln_bwd_kernel<true>, dim3(grid), dim3(256), 0, s, nullptr, a, xhat, rstd, gamma, R,
                     drop_threshold(p_drop), 1.0f / (1.0f - p_drop), seed, (uint32_t)salt,
                     reinterpret_cast<bf16 *>(da), ws, dout, hmask, hw, beta, hpart);
  if (defer) {
    FS2_CHECK_LAUNCH();
    return FS2_OK;
  }
  hipLaunchKernelGGL(ln_finish_kernel, dim3(3 * kD / 64), dim3(256), 0, s, ws, grid, dgamma, dbeta, dbias, accumulate);
  FS2_CHECK_LAUNCH();
  fs2_reduce_batch rb{};
  rb.n = 1;
  rb.d[0].part = hpart;
  rb.d[0].M = kD + 4;
  rb.d[0].S = grid;
  rb.d[0].kind = 2;
  rb.d[0].split = kD;
  rb.d[0].accumulate = accumulate;
  rb.d[0].out0 = dhw;
  rb.d[0].out1 = dhb;
  return fs2_reduce_batch_launch(&rb, stream);
}

extern "C" int fs2_embedding_bwd(const int64_t *tokens, int64_t n, const float *dy, int64_t dy_row_stride, int V,
                                 int D, int padding_idx, float *out, int accumulate, fs2_stream_t stream) {
  if (tokens == nullptr || out == nullptr || (n > 0 && dy == nullptr)) return FS2_EINVAL;
  if (n < 0 || V <= 0 || D <= 0 || D > 256 || dy_row_stride < D) return FS2_EINVAL;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)V), dim3(256), 0, as_stream(stream), tokens, n, dy,
                     dy_row_stride, D, padding_idx, out, accumulate);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int64_t fs2_colsum_ws_bytes(int N) { return 64LL * ((N + 255) / 256 * 256) * (int64_t)sizeof(float); }

extern "C" int fs2_colsum(const void *x, int dtype, int64_t R, int N, int64_t row_stride, float *out, int accumulate,
                          float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (x == nullptr || out == nullptr || ws == nullptr) return FS2_EINVAL;
  if (R < 0 || N <= 0 || (N & 3) || row_stride < N || (row_stride & 3)) return FS2_EINVAL;
  if (ws_bytes < fs2_colsum_ws_bytes(N)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  int chunks = (int)((R + 127) / 128);
  if (chunks > 64) chunks = 64;
  if (chunks < 1) chunks = 1;
  const int rpc = (int)((R + chunks - 1) / chunks);
  dim3 g1((unsigned)((N + 255) / 256), (unsigned)chunks);
  if (dtype == FS2_F32)
    hipLaunchKernelGGL(colsum_part_kernel<float>, g1, dim3(256), 0, s, reinterpret_cast<const float *>(x), R, N,
                       row_stride, rpc, ws);
  else if (dtype == FS2_BF16)
    hipLaunchKernelGGL(colsum_part_kernel<bf16>, g1, dim3(256), 0, s, reinterpret_cast<const bf16 *>(x), R, N,
                       row_stride, rpc, ws);
  else
    return FS2_EUNSUPPORTED;
  hipLaunchKernelGGL(colsum_finish_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, ws, chunks, N, out,
                     accumulate);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// Conv1d / Linear weight gradient (Conv1dFn.backward's dW, training.py):
//   dW[n][c][k] = sum_{b, t} dy[b, t, n] * x[b, t + k - pad, c]     (x zero outside [0, T) per sequence)
// and optionally db[n] = sum_{b, t} dy[b, t, n]. No unfolded copy of x: per 32-row chunk of one
// sequence the block stages dy [32 x NB] and the x window [32 + KS - 1 rows x CB] in LDS (plain
// rows, chunk-XOR swizzled), and both MFMA operands come out of them with ds_read_b64_tr_b16 (the
// reduction index m is the row index of both tiles). The KS taps share one x window: a lane reads
// rows 8g .. 8g + 7 + KS - 1 of its column once and forms tap k's 8-row fragment from registers
// (even k: a dword offset; odd k: v_alignbit of neighbouring dwords).
// Block = 4 waves stacked along n (wave tile 16*WN x 64*WCB, all KS taps in accumulators); grid
// (n tiles x c tiles, S row splits); split partials part[s][k][n][c] are summed in order by
// wgrad_reduce_kernel (deterministic; optionally accumulated into an existing gradient).
// ---------------------------------------------------------------------------------------------
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));

struct WgArgs {
  const void *dy;
  int64_t dys;
  const bf16 *x;
  int64_t xs;
  float *part;
  float *pbias;
  int B, T, N, C, pad, S, tiles_c, CT;  // CT = 32-row chunks per sequence
};

// 128-byte LDS rows (64 bf16), 16-byte chunk XOR: conflict-free ds_read_b64_tr_b16 for 8-row
// separated lane groups at any base row (exhaustive search over linear XOR maps).
__device__ __forceinline__ int wg_off(int row, int colbyte) {
  const int ch = (colbyte >> 4) ^ (((row >> 1) & 1) << 1) ^ (((row >> 3) & 1) << 2);
  return row * 128 + (ch << 4) + (colbyte & 15);
}

__device__ __forceinline__ uint2 tr_read(const char *lds_base, int off) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(lds_base + off));
  uint2 r;
  __builtin_memcpy(&r, &v, 8);
  return r;
}

__device__ __forceinline__ uint4 f32x8_to_bf16(float4 a, float4 b) {
  float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
  uint4 r;
  __builtin_memcpy(&r, &o, 16);
  return r;
}

template <int KS, int WN, int WCB, bool DYF32>
__global__ __launch_bounds__(256, 1) void wgrad_kernel(WgArgs a) {
  constexpr int NB = 64 * WN;            // n columns per block
  constexpr int CB = 64 * WCB;           // c columns per block
  constexpr int NR = (KS + 7 + 3) / 4;   // 4-row transposed reads per x fragment group
  constexpr int XR = 24 + 4 * NR;        // x window rows held in LDS (>= 32 + KS - 1)
  constexpr int DY_BYTES = WN * 32 * 128;
  constexpr int X_BYTES = WCB * XR * 128;
  constexpr int BUF = DY_BYTES + X_BYTES;
  constexpr int DY_LD = NB / 8 * 32 / 256 > 0 ? NB / 8 * 32 / 256 : 1;  // 16-byte dy loads per thread
  constexpr int X_CHUNKS = XR * CB / 8;
  constexpr int X_LD = (X_CHUNKS + 255) / 256;
  constexpr int DYW = DYF32 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int tile = blockIdx.x, s = blockIdx.y;
  const int n0 = (tile / a.tiles_c) * NB, c0 = (tile % a.tiles_c) * CB;
  const int Q = a.B * a.CT;
  const bool do_bias = a.pbias != nullptr && (tile % a.tiles_c) == 0;

  uint4 rdy[DY_LD][DYW];
  uint4 rx[X_LD];
  float bsum[DY_LD][8];
#pragma unroll
  for (int i = 0; i < DY_LD; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) bsum[i][q] = 0.f;

  auto load = [&](int q) {
    const int b = q / a.CT, t0 = (q - b * a.CT) * 32;
#pragma unroll
    for (int i = 0; i < DY_LD; ++i) {
      const int e = tid + 256 * i;              // 16-byte chunk: row e / (NB/8), col group e % (NB/8)
      const int r = e / (NB / 8), cg = e % (NB / 8);
      const int t = t0 + r, n = n0 + cg * 8;
      if (t < a.T && n < a.N) {
        const int64_t row = (int64_t)b * a.T + t;
        if constexpr (DYF32) {
          const float4 *p = reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(a.dy) + row * a.dys + n);
          float4 v0 = p[0], v1 = p[1];
          __builtin_memcpy(&rdy[i][0], &v0, 16);
          __builtin_memcpy(&rdy[i][1], &v1, 16);
        } else {
          rdy[i][0] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16 *>(a.dy) + row * a.dys + n);
        }
      } else {
#pragma unroll
        for (int h = 0; h < DYW; ++h) rdy[i][h] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < X_LD; ++i) {
      const int e = tid + 256 * i;
      const int r = e / (CB / 8), cg = e % (CB / 8);
      const int t = t0 - a.pad + r, c = c0 + cg * 8;
      rx[i] = make_uint4(0, 0, 0, 0);
      if (e < X_CHUNKS && r < 32 + KS - 1 && t >= 0 && t < a.T && c < a.C)
        rx[i] = *reinterpret_cast<const uint4 *>(a.x + ((int64_t)b * a.T + t) * a.xs + c);
    }
  };
  auto store = [&](int buf) {
    char *base = lds + buf * BUF;
#pragma unroll
    for (int i = 0; i < DY_LD; ++i) {
      const int e = tid + 256 * i;
      const int r = e / (NB / 8), cg = e % (NB / 8);
      uint4 v;
      if constexpr (DYF32) {
        float4 v0, v1;
        __builtin_memcpy(&v0, &rdy[i][0], 16);
        __builtin_memcpy(&v1, &rdy[i][1], 16);
        if (do_bias) {
          bsum[i][0] += v0.x; bsum[i][1] += v0.y; bsum[i][2] += v0.z; bsum[i][3] += v0.w;
          bsum[i][4] += v1.x; bsum[i][5] += v1.y; bsum[i][6] += v1.z; bsum[i][7] += v1.w;
        }
        v = f32x8_to_bf16(v0, v1);
      } else {
        v = rdy[i][0];
        if (do_bias) {
          const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            bsum[i][2 * h] += __uint_as_float(wd[h] << 16);
            bsum[i][2 * h + 1] += __uint_as_float(wd[h] & 0xffff0000u);
          }
        }
      }
      *reinterpret_cast<uint4 *>(base + (cg >> 3) * 32 * 128 + wg_off(r, (cg & 7) * 16)) = v;
    }
#pragma unroll
    for (int i = 0; i < X_LD; ++i) {
      const int e = tid + 256 * i;
      if (e < X_CHUNKS) {
        const int r = e / (CB / 8), cg = e % (CB / 8);
        *reinterpret_cast<uint4 *>(base + DY_BYTES + (cg >> 3) * XR * 128 + wg_off(r, (cg & 7) * 16)) = rx[i];
      }
    }
  };

  f32x4 acc[KS][WN][4 * WCB];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int wn = 0; wn < WN; ++wn)
#pragma unroll
      for (int j = 0; j < 4 * WCB; ++j) acc[k][wn][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int q = s;
  int cur = 0;
  if (q < Q) {
    load(q);
    store(0);
  }
  __syncthreads();
  // lane's transposed-read address parts: row q4 = li >> 2 of a 4-row block, 8-byte column piece
  const int trow = 8 * g + (li >> 2), tcol = 8 * (li & 3);
  for (; q < Q; q += a.S) {
    const bool more = q + a.S < Q;
    if (more) load(q + a.S);
    const char *base = lds + cur * BUF;
    bf16x8 A[WN];
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) {
      const int nl = w * 16 * WN + wn * 16;  // wave's n block within the tile
      const char *sb = base + (nl >> 6) * 32 * 128;
      const uint2 lo = tr_read(sb, wg_off(trow, (nl & 63) * 2 + tcol));
      const uint2 hi = tr_read(sb, wg_off(trow + 4, (nl & 63) * 2 + tcol));
      uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
      __builtin_memcpy(&A[wn], &u, 16);
    }
#pragma unroll
    for (int j = 0; j < 4 * WCB; ++j) {
      const char *xb = base + DY_BYTES + (j >> 2) * XR * 128;
      uint32_t xw[2 * NR];
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        const uint2 v = tr_read(xb, wg_off(trow + 4 * u, (j & 3) * 32 + tcol));
        xw[2 * u] = v.x;
        xw[2 * u + 1] = v.y;
      }
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        uint32_t f[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
          f[d] = (k & 1) ? __builtin_amdgcn_alignbit(xw[(k + 1) / 2 + d], xw[(k - 1) / 2 + d], 16) : xw[k / 2 + d];
        bf16x8 Bf;
        __builtin_memcpy(&Bf, f, 16);
#pragma unroll
        for (int wn = 0; wn < WN; ++wn)
          acc[k][wn][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[wn], Bf, acc[k][wn][j], 0, 0, 0);
      }
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // split partial: part[s][k][n][c]
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int wn = 0; wn < WN; ++wn)
#pragma unroll
      for (int j = 0; j < 4 * WCB; ++j) {
        const int c = c0 + 16 * j + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + w * 16 * WN + wn * 16 + 4 * g + r;
          if (n < a.N && c < a.C) a.part[(((int64_t)s * KS + k) * a.N + n) * a.C + c] = acc[k][wn][j][r];
        }
      }
  if (do_bias) {  // rows of the block's dy loads -> per-column sums, in a fixed order
    constexpr int RPP = 256 / (NB / 8);  // rows per load pass
    float *red = reinterpret_cast<float *>(lds);
#pragma unroll
    for (int i = 0; i < DY_LD; ++i) {
      const int e = tid + 256 * i;
      const int r = e / (NB / 8), cg = e % (NB / 8);
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) red[((i * RPP) + (r % RPP)) * NB + cg * 8 + qq] = bsum[i][qq];
    }
    __syncthreads();
    if (tid < NB) {
      float sacc = 0.f;
      for (int r = 0; r < DY_LD * RPP; ++r) sacc += red[r * NB + tid];
      if (n0 + tid < a.N) a.pbias[(int64_t)s * a.N + n0 + tid] = sacc;
    }
  }
}

// out[n][c][k] (+)= sum over splits of part[s][k][n][c]; rows n >= split go to the next output
// (parts of one gradient that are separate parameters: Q | K | V)
struct WgOut {
  float *dw[3];
  float *db[3];
  int split;
};

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float *__restrict__ part, int S, int KS, int N, int C,
                                                           WgOut o, int accumulate) {
  const int64_t NC = (int64_t)N * C;
  const int64_t e = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);  // (k, n, c) of part's rows
  const float sacc = parts_col_sum(part, S, NC * KS, e);
  if (threadIdx.x >= 64 || e >= NC * KS) return;
  const int k = (int)(e / NC);
  const int64_t nc = e - (int64_t)k * NC;
  const int n = (int)(nc / C), which = n / o.split;
  float *dst = o.dw[which] + (nc - (int64_t)which * o.split * C) * KS + k;
  *dst = accumulate ? *dst + sacc : sacc;
}

__global__ __launch_bounds__(256) void bias_reduce_kernel(const float *__restrict__ part, int S, int N, WgOut o,
                                                          int accumulate) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const float s = parts_col_sum(part, S, N, n);
  if (threadIdx.x >= 64 || n >= N) return;
  const int which = n / o.split;
  float *dst = o.db[which] + (n - which * o.split);
  *dst = accumulate ? *dst + s : s;
}

template <int KS, int WN, int WCB>
void wgrad_launch(const WgArgs &a, bool dy_f32, int tiles, hipStream_t s) {
  if (dy_f32)
    hipLaunchKernelGGL((wgrad_kernel<KS, WN, WCB, true>), dim3(tiles, a.S), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((wgrad_kernel<KS, WN, WCB, false>), dim3(tiles, a.S), dim3(256), 0, s, a);
}

int wgrad_splits(int tiles, int Q, int KS_) {
  // enough workgroups to fill the chip, few enough splits that the partials stay small (each
  // split adds a full f32 copy of dW to write and re-read)
  // KS == 1 (dW of Q|K|V, fc, w_2, mel_linear: <= 1 MB outputs): up to 32 splits for ~512
  // workgroups; wide-tap convs (FFN w_1: a 9.4 MB dW) at most 8 splits for ~256
  const int target = KS_ == 1 ? 512 : 256, cap = KS_ == 1 ? 16 : 8;
  int S = (target + tiles - 1) / tiles;
  if (S > Q) S = Q;
  if (S > cap) S = cap;
  return S < 1 ? 1 : S;
}

}  // namespace

extern "C" int fs2_conv_wgrad_splits(int B, int T, int N, int C, int KS) {
  if (B <= 0 || T <= 0 || N <= 0 || C <= 0 || KS <= 0) return 1;
  const int WN = KS == 1 ? 2 : 1, WCB = KS == 1 ? 2 : 1;
  const int tiles = ((N + 64 * WN - 1) / (64 * WN)) * ((C + 64 * WCB - 1) / (64 * WCB));
  return wgrad_splits(tiles, B * ((T + 31) / 32), KS);
}

extern "C" int64_t fs2_conv_wgrad_ws_bytes(int B, int T, int N, int C, int KS) {
  if (B <= 0 || T <= 0 || N <= 0 || C <= 0 || KS <= 0) return 0;
  const int WN = KS == 1 ? 2 : 1, WCB = KS == 1 ? 2 : 1;
  const int tiles = ((N + 64 * WN - 1) / (64 * WN)) * ((C + 64 * WCB - 1) / (64 * WCB));
  const int S = wgrad_splits(tiles, B * ((T + 31) / 32), KS);
  return ((int64_t)S * KS * N * C + (int64_t)S * N) * (int64_t)sizeof(float);
}

extern "C" int fs2_conv_wgrad(const void *dy, int dy_dtype, int64_t dy_row_stride, const void *x,
                              int64_t x_row_stride, int B, int T, int N, int C, int KS, int pad, float *dw,
                              float *db, int accumulate, int split_rows, float *dw1, float *dw2, float *db1,
                              float *db2, int defer, float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dy == nullptr || x == nullptr || (dw == nullptr && !defer) || ws == nullptr) return FS2_EINVAL;
  WgOut o;
  o.dw[0] = dw, o.dw[1] = dw1, o.dw[2] = dw2;
  o.db[0] = db, o.db[1] = db1, o.db[2] = db2;
  o.split = N;
  if (split_rows > 0) {  // N = 2 or 3 equal row parts, each its own tensor
    if (N % split_rows || N / split_rows > 3 || N / split_rows < 2) return FS2_EINVAL;
    for (int i = 1; i < N / split_rows; ++i)
      if (o.dw[i] == nullptr || (db != nullptr && o.db[i] == nullptr)) return FS2_EINVAL;
    o.split = split_rows;
  }
  if (B < 0 || T < 0 || N <= 0 || C <= 0 || (N & 7) || (C & 7) || pad < 0 || pad >= KS) return FS2_EINVAL;
  if (dy_row_stride < N || x_row_stride < C || (dy_row_stride & 7) || (x_row_stride & 7)) return FS2_EINVAL;
  if (dy_dtype != FS2_BF16 && dy_dtype != FS2_F32) return FS2_EUNSUPPORTED;
  if (KS != 1 && KS != 3 && KS != 5 && KS != 9) return FS2_EUNSUPPORTED;
  hipStream_t s = as_stream(stream);
  if ((int64_t)B * T == 0) {
    if (defer) {  // the batch reduction sums zero partials
      (void)hipMemsetAsync(ws, 0, (size_t)fs2_conv_wgrad_ws_bytes(B > 0 ? B : 1, T > 0 ? T : 1, N, C, KS), s);
      return FS2_OK;
    }
    if (!accumulate)
      for (int i = 0; i * o.split < N; ++i) {
        (void)hipMemsetAsync(o.dw[i], 0, (size_t)o.split * C * KS * sizeof(float), s);
        if (db != nullptr) (void)hipMemsetAsync(o.db[i], 0, (size_t)o.split * sizeof(float), s);
      }
    return FS2_OK;
  }
  if (ws_bytes < fs2_conv_wgrad_ws_bytes(B, T, N, C, KS)) return FS2_EINVAL;
  const int WN = KS == 1 ? 2 : 1, WCB = KS == 1 ? 2 : 1;
  WgArgs a;
  a.dy = dy;
  a.dys = dy_row_stride;
  a.x = reinterpret_cast<const bf16 *>(x);
  a.xs = x_row_stride;
  a.B = B;
  a.T = T;
  a.N = N;
  a.C = C;
  a.pad = pad;
  a.CT = (T + 31) / 32;
  a.tiles_c = (C + 64 * WCB - 1) / (64 * WCB);
  const int tiles = ((N + 64 * WN - 1) / (64 * WN)) * a.tiles_c;
  a.S = wgrad_splits(tiles, B * a.CT, KS);
  a.part = ws;
  a.pbias = db != nullptr ? ws + (int64_t)a.S * KS * N * C : nullptr;
  const bool f32 = dy_dtype == FS2_F32;
  switch (KS) {
    case 1: wgrad_launch<1, 2, 2>(a, f32, tiles, s); break;
    case 3: wgrad_launch<3, 1, 1>(a, f32, tiles, s); break;
    case 5: wgrad_launch<5, 1, 1>(a, f32, tiles, s); break;
    default: wgrad_launch<9, 1, 1>(a, f32, tiles, s); break;
  }
  if (defer) {  // partials left in ws for fs2_reduce_batch
    FS2_CHECK_LAUNCH();
    return FS2_OK;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(((int64_t)N * C * KS + 63) / 64)), dim3(256), 0, s, ws, a.S,
                     KS, N, C, o, accumulate);
  if (db != nullptr)
    hipLaunchKernelGGL(bias_reduce_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, a.pbias, a.S, N, o,
                       accumulate);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// All of a step's MFMA weight images in ONE launch (the FFT blocks' Q|K|V, fc, w_1, w_2): per
// f32 weight [N][C][KS] (nn.Conv1d; Linear KS = 1) the forward image fwd bf16 [N_tot][KS][C] at row
// n_off and the input-gradient image tr bf16 [C][KS][N_tot] (taps flipped, W transposed) at
// column n_off; f32 descriptors copy a vector (Q|K|V biases) into one f32 buffer. 32 x 32 (n, c)
// tiles; the transposed image goes through LDS so both stores are coalesced.
// ---------------------------------------------------------------------------------------------
namespace {

__global__ __launch_bounds__(256) void pack_train_kernel(const fs2_pack_desc *__restrict__ descs, int nd) {
  __shared__ float t[9][32][33];
  int i = 0;
  for (int j = 1; j < nd; ++j)
    if (descs[j].blk0 <= (int)blockIdx.x) i = j;
  const fs2_pack_desc d = descs[i];
  const int tile = blockIdx.x - d.blk0;
  const int tn = tile / d.tiles_c, tc = tile - tn * d.tiles_c;
  const int cl = threadIdx.x & 31, nl0 = threadIdx.x >> 5;
  const int c = tc * 32 + cl;
  if (d.f32_copy) {  // vector copy: N elements at n_off
    const int n = tile * 256 + threadIdx.x;
    if (n < d.N) reinterpret_cast<float *>(d.fwd)[d.n_off + n] = d.src[n];
    return;
  }
  const int KS = d.KS;
  for (int r = 0; r < 4; ++r) {
    const int nl = nl0 + 8 * r, n = tn * 32 + nl;
    if (n < d.N && c < d.C) {
      const float *s = d.src + ((int64_t)n * d.C + c) * KS;
      for (int k = 0; k < KS; ++k) {
        const float v = s[k];
        if (d.fwd != nullptr) reinterpret_cast<bf16 *>(d.fwd)[((int64_t)(d.n_off + n) * KS + k) * d.C_tot + c] = (bf16)v;
        t[k][nl][cl] = v;
      }
    }
  }
  if (d.tr == nullptr) return;
  __syncthreads();
  const int nl = threadIdx.x & 31, cl0 = threadIdx.x >> 5;
  const int n = tn * 32 + nl;
  for (int r = 0; r < 4; ++r) {
    const int clr = cl0 + 8 * r, cc = tc * 32 + clr;
    if (n < d.N && cc < d.C)
      for (int k = 0; k < KS; ++k)
        reinterpret_cast<bf16 *>(d.tr)[((int64_t)cc * KS + k) * d.N_tot + d.n_off + n] = (bf16)t[KS - 1 - k][nl][clr];
  }
}

}  // namespace

extern "C" int fs2_pack_train_plan(fs2_pack_desc *descs, int nd, int *blocks) {
  if (descs == nullptr || nd <= 0 || blocks == nullptr) return FS2_EINVAL;
  int blk = 0;
  for (int i = 0; i < nd; ++i) {
    fs2_pack_desc &d = descs[i];
    if (d.src == nullptr || (d.fwd == nullptr && d.tr == nullptr)) return FS2_EINVAL;
    if (d.f32_copy) {
      if (d.N <= 0 || d.tr != nullptr) return FS2_EINVAL;
      d.tiles_c = 1;
      d.blk0 = blk;
      blk += (d.N + 255) / 256;
      continue;
    }
    if (d.C_tot == 0) d.C_tot = d.C;
    if (d.N <= 0 || d.C <= 0 || d.KS < 1 || d.KS > 9 || d.n_off < 0 || d.n_off + d.N > d.N_tot || d.C_tot < d.C)
      return FS2_EINVAL;
    d.tiles_c = (d.C + 31) / 32;
    d.blk0 = blk;
    blk += ((d.N + 31) / 32) * d.tiles_c;
  }
  *blocks = blk;
  return FS2_OK;
}

extern "C" int fs2_pack_train(const fs2_pack_desc *descs_dev, int nd, int blocks, fs2_stream_t stream) {
  if (descs_dev == nullptr || nd <= 0 || blocks <= 0) return FS2_EINVAL;
  hipLaunchKernelGGL(pack_train_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), descs_dev, nd);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// FastSpeech2Loss (model/loss.py:5-92): the five masked means and their total in one reduction
// (fixed-order partials: deterministic) and every prediction's gradient in one elementwise pass.
//   mel / postnet: L1 over the valid frames' n_mel channels; pitch / energy / log-duration: MSE
//   over their masks (log_d target = log(d + 1)); empty masks give NaN, as masked_select().mean().
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kLossBlocks = 256;
constexpr int kLossQ = 9;  // s_mel, s_post, n_rows, s_p, n_p, s_e, n_e, s_d, n_d

__global__ __launch_bounds__(256) void loss_part_kernel(fs2_loss_args a, float *__restrict__ part) {
  __shared__ float red[4][kLossQ];
  float q[kLossQ];
#pragma unroll
  for (int i = 0; i < kLossQ; ++i) q[i] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c4n = a.n_mel / 4;
  const int64_t nmel = (int64_t)a.B * a.T * c4n;
  for (int64_t i = g0; i < nmel; i += stride) {
    const int64_t row = i / c4n;
    const int c = (int)(i - row * c4n) * 4;
    if (!a.mel_valid[row]) continue;
    const int64_t b = row / a.T, t = row - b * a.T;
    float m[4], p[4], tg[4];
    load4(a.mel + row * a.n_mel + c, m);
    load4(a.postnet + row * a.n_mel + c, p);
    load4(a.mel_tgt + b * a.tgt_bs + t * a.tgt_ts + c, tg);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[0] += fabsf(m[k] - tg[k]);
      q[1] += fabsf(p[k] - tg[k]);
    }
    if (c == 0) q[2] += 1.f;
  }
  for (int64_t i = g0; i < a.n_p; i += stride)
    if (a.p_mask[i]) {
      const float d = a.p_pred[i] - a.p_tgt[i];
      q[3] += d * d;
      q[4] += 1.f;
    }
  for (int64_t i = g0; i < a.n_e; i += stride)
    if (a.e_mask[i]) {
      const float d = a.e_pred[i] - a.e_tgt[i];
      q[5] += d * d;
      q[6] += 1.f;
    }
  for (int64_t i = g0; i < a.n_d; i += stride)
    if (a.d_mask[i]) {
      const float d = a.logd_pred[i] - logf((float)a.d_tgt[i] + 1.0f);
      q[7] += d * d;
      q[8] += 1.f;
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kLossQ; ++i) {
    const float v = wave_sum(q[i]);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kLossQ)
    part[(int64_t)blockIdx.x * kLossQ + threadIdx.x] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// out[0..5] = total, mel, postnet, pitch, energy, duration; stats[0..3] = n_mel_elems, n_p, n_e, n_d
__global__ __launch_bounds__(256) void loss_finish_kernel(const float *__restrict__ part, int blocks, int n_mel,
                                                          float *__restrict__ out, float *__restrict__ stats) {
  __shared__ float sv[kLossQ];
  const float v = parts_col_sum(part, blocks, kLossQ, threadIdx.x & 63);
  if (threadIdx.x < kLossQ) sv[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float *s = sv;
    const float nm = s[2] * (float)n_mel;
    const float mel = s[0] / nm, post = s[1] / nm, pl = s[3] / s[4], el = s[5] / s[6], dl = s[7] / s[8];
    out[1] = mel;
    out[2] = post;
    out[3] = pl;
    out[4] = el;
    out[5] = dl;
    out[0] = (((mel + post) + dl) + pl) + el;  // model/loss.py:84-86 order
    stats[0] = nm;
    stats[1] = s[4];
    stats[2] = s[6];
    stats[3] = s[8];
  }
}

// gradients: g[0..5] upstream of (total, mel, postnet, pitch, energy, duration); stats = out[6..9]
__global__ __launch_bounds__(256) void loss_bwd_kernel(fs2_loss_args a, const float *__restrict__ g,
                                                       const float *__restrict__ stats, float *__restrict__ d_mel,
                                                       float *__restrict__ d_post, float *__restrict__ d_p,
                                                       float *__restrict__ d_e, float *__restrict__ d_logd) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const float gt = g[0];
  const float km = (gt + g[1]) / stats[0], kp = (gt + g[2]) / stats[0];
  const int c4n = a.n_mel / 4;
  const int64_t nmel = (int64_t)a.B * a.T * c4n;
  for (int64_t i = g0; i < nmel; i += stride) {
    const int64_t row = i / c4n;
    const int c = (int)(i - row * c4n) * 4;
    float dm[4] = {0.f, 0.f, 0.f, 0.f}, dp[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.mel_valid[row]) {
      const int64_t b = row / a.T, t = row - b * a.T;
      float m[4], p[4], tg[4];
      load4(a.mel + row * a.n_mel + c, m);
      load4(a.postnet + row * a.n_mel + c, p);
      load4(a.mel_tgt + b * a.tgt_bs + t * a.tgt_ts + c, tg);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float e1 = m[k] - tg[k], e2 = p[k] - tg[k];
        dm[k] = e1 > 0.f ? km : (e1 < 0.f ? -km : 0.f);
        dp[k] = e2 > 0.f ? kp : (e2 < 0.f ? -kp : 0.f);
      }
    }
    store4(d_mel + row * a.n_mel + c, dm);
    store4(d_post + row * a.n_mel + c, dp);
  }
  const float kpi = 2.f * (gt + g[3]) / stats[1], ke = 2.f * (gt + g[4]) / stats[2],
              kd = 2.f * (gt + g[5]) / stats[3];
  for (int64_t i = g0; i < a.n_p; i += stride) d_p[i] = a.p_mask[i] ? kpi * (a.p_pred[i] - a.p_tgt[i]) : 0.f;
  for (int64_t i = g0; i < a.n_e; i += stride) d_e[i] = a.e_mask[i] ? ke * (a.e_pred[i] - a.e_tgt[i]) : 0.f;
  for (int64_t i = g0; i < a.n_d; i += stride)
    d_logd[i] = a.d_mask[i] ? kd * (a.logd_pred[i] - logf((float)a.d_tgt[i] + 1.0f)) : 0.f;
}

int loss_check(const fs2_loss_args *a) {
  if (a == nullptr || a->mel == nullptr || a->postnet == nullptr || a->mel_tgt == nullptr || a->mel_valid == nullptr ||
      a->p_pred == nullptr || a->p_tgt == nullptr || a->p_mask == nullptr || a->e_pred == nullptr ||
      a->e_tgt == nullptr || a->e_mask == nullptr || a->logd_pred == nullptr || a->d_tgt == nullptr ||
      a->d_mask == nullptr)
    return FS2_EINVAL;
  if (a->B < 0 || a->T < 0 || a->n_mel <= 0 || (a->n_mel & 3) || a->n_p < 0 || a->n_e < 0 || a->n_d < 0 ||
      (a->tgt_ts & 3) || (a->tgt_bs & 3))
    return FS2_EINVAL;
  return FS2_OK;
}

}  // namespace

extern "C" int64_t fs2_loss_ws_bytes(void) { return (int64_t)kLossBlocks * kLossQ * (int64_t)sizeof(float); }

extern "C" int fs2_loss_fwd(const fs2_loss_args *a, float *out, float *stats, float *ws, int64_t ws_bytes,
                            fs2_stream_t stream) {
  const int st = loss_check(a);
  if (st != FS2_OK) return st;
  if (out == nullptr || stats == nullptr || ws == nullptr || ws_bytes < fs2_loss_ws_bytes()) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(loss_part_kernel, dim3(kLossBlocks), dim3(256), 0, s, *a, ws);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, s, ws, kLossBlocks, a->n_mel, out, stats);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_loss_bwd(const fs2_loss_args *a, const float *grad_out, const float *stats, float *d_mel,
                            float *d_postnet, float *d_pitch, float *d_energy, float *d_logd, fs2_stream_t stream) {
  const int st = loss_check(a);
  if (st != FS2_OK) return st;
  if (grad_out == nullptr || stats == nullptr || d_mel == nullptr || d_postnet == nullptr || d_pitch == nullptr ||
      d_energy == nullptr || d_logd == nullptr)
    return FS2_EINVAL;
  const int64_t work = (int64_t)a->B * a->T * (a->n_mel / 4);
  int64_t blocks = (work + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  hipLaunchKernelGGL(loss_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), *a, grad_out, stats,
                     d_mel, d_postnet, d_pitch, d_energy, d_logd);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// PostNet layer in train mode (transformer/Layers.py:92-137, training.py): BatchNorm1d on batch
// statistics over all B*T frames (running stats updated with momentum, unbiased variance), tanh
// (layers 0..3), F.dropout(0.5). Statistics: per block a two-pass (mean, M2) over its row chunk,
// combined in block order with Chan's formula (deterministic, no E[z^2] - E[z]^2 cancellation).
// The backward recomputes zhat and tanh from z and regenerates the dropout bits.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kBnBlocks = 256;

struct BnGeom {
  int G, RPI, cg, rsub;  // column groups of 4, rows per iteration, this thread's group / row slot
  bool active;
};

__device__ __forceinline__ BnGeom bn_geom(int C) {
  BnGeom g;
  g.G = C >> 2;
  g.RPI = 256 / g.G;
  g.cg = threadIdx.x % g.G;
  g.rsub = threadIdx.x / g.G;
  g.active = g.rsub < g.RPI;
  return g;
}

// reduce v[4] (this thread's 4 columns) over the RPI row slots through LDS; result for columns
// [4*cg, 4*cg+4) left in v on threads with rsub == 0
__device__ __forceinline__ void bn_row_reduce(float *red, const BnGeom &g, int C, float v[4]) {
  __syncthreads();
  if (g.active)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[g.rsub * C + g.cg * 4 + q] = v[q];
  __syncthreads();
  if (g.active && g.rsub == 0)
    for (int r = 1; r < g.RPI; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += red[r * C + g.cg * 4 + q];
}

// part[blk][c][2] = (sum (z - K_c), sum (z - K_c)^2) over the block's rows, K_c = z[0][c]: shifted
// sums (no E[z^2] - E[z]^2 cancellation for |mean| >> std), added in a fixed order by the finish
__global__ __launch_bounds__(256) void bn_stats_part_kernel(const float *__restrict__ z, int64_t R, int C, int rpb,
                                                            float *__restrict__ part) {
  extern __shared__ float red[];
  const BnGeom g = bn_geom(C);
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < R ? r0 + rpb : R;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.active) {
    float K[4];
    load4(z + g.cg * 4, K);
    for (int64_t r = r0 + g.rsub; r < r1; r += g.RPI) {
      float v[4];
      load4(z + r * C + g.cg * 4, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = v[q] - K[q];
        s1[q] += d;
        s2[q] += d * d;
      }
    }
  }
  bn_row_reduce(red, g, C, s1);
  bn_row_reduce(red, g, C, s2);
  if (g.active && g.rsub == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float *p = part + ((int64_t)blockIdx.x * C + g.cg * 4 + q) * 2;
      p[0] = s1[q];
      p[1] = s2[q];
    }
}

__global__ __launch_bounds__(256) void bn_stats_finish_kernel(const float *__restrict__ z, int64_t R,
                                                              const float *__restrict__ part, int blocks, int C,
                                                              float eps, float momentum, float *running_mean,
                                                              float *running_var, float *__restrict__ mean_out,
                                                              float *__restrict__ rstd_out) {
  __shared__ float sv[2][64];
  const int64_t col = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);  // c * 2 + j
  const float v = parts_col_sum(part, blocks, 2LL * C, col);
  if (threadIdx.x < 64) sv[col & 1][threadIdx.x >> 1] = v;  // (sum, sum of squares) of channel col / 2
  __syncthreads();
  if (threadIdx.x >= 32) return;
  const int c = blockIdx.x * 32 + threadIdx.x;
  if (c >= C) return;
  const double n = (double)R, m1 = (double)sv[0][threadIdx.x] / n;
  const double var = fmax((double)sv[1][threadIdx.x] / n - m1 * m1, 0.0);
  const float mean = z[c] + (float)m1;
  mean_out[c] = mean;
  rstd_out[c] = rsqrtf((float)var + eps);
  if (running_mean != nullptr) {
    running_mean[c] = (1.0f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.0f - momentum) * running_var[c] + momentum * (float)(var * n / (n > 1.0 ? n - 1.0 : 1.0));
  }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(const float *__restrict__ z, int64_t R, int C,
                                                       const float *__restrict__ mean, const float *__restrict__ rstd,
                                                       const float *__restrict__ gamma, const float *__restrict__ beta,
                                                       int use_tanh, uint32_t thr, float scale, const int64_t *seed,
                                                       uint32_t salt, const float *__restrict__ residual,
                                                       bf16 *__restrict__ y_bf, float *__restrict__ y_f32) {
  const uint32_t key = drop_key(seed, salt);
  const int64_t n4 = R * (C >> 2);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / (C >> 2);
    const int c = (int)(i - row * (C >> 2)) * 4;
    float v[4], mu[4], rs[4], g[4], b[4];
    load4(z + row * C + c, v);
    load4(mean + c, mu);
    load4(rstd + c, rs);
    load4(gamma + c, g);
    load4(beta + c, b);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = (v[q] - mu[q]) * rs[q] * g[q] + b[q];
      if (use_tanh) v[q] = tanhf(v[q]);
    }
    if (thr != 0) {
      const unsigned k = keep4(key, (uint32_t)(row * C + c), thr);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ((k >> q) & 1) ? v[q] * scale : 0.0f;
    }
    if (residual != nullptr) {
      float r[4];
      load4(residual + row * C + c, r);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += r[q];
    }
    if (y_bf != nullptr) store4(y_bf + row * C + c, v);
    if (y_f32 != nullptr) store4(y_f32 + row * C + c, v);
  }
}

// backward pass 1: per block, per column: sum dpre and sum dpre * zhat, dpre = dy * keep * scale * tanh'
__device__ __forceinline__ void bn_dpre(const float *dy, const float *z, int64_t row, int C, int c, const float *mu,
                                        const float *rs, const float *g, const float *b, int use_tanh, uint32_t key,
                                        uint32_t thr, float scale, float dp[4], float zh[4]) {
  float d[4], v[4];
  load4(dy + row * C + c, d);
  load4(z + row * C + c, v);
  unsigned k = 0xf;
  if (thr != 0) k = keep4(key, (uint32_t)(row * C + c), thr);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    zh[q] = (v[q] - mu[q]) * rs[q];
    float t = ((k >> q) & 1) ? d[q] * scale : 0.0f;
    if (use_tanh) {
      const float a = tanhf(zh[q] * g[q] + b[q]);
      t *= 1.0f - a * a;
    }
    dp[q] = t;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_part_kernel(const float *__restrict__ dy, const float *__restrict__ z,
                                                          int64_t R, int C, int rpb, const float *__restrict__ mean,
                                                          const float *__restrict__ rstd, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta, int use_tanh, uint32_t thr,
                                                          float scale, const int64_t *seed, uint32_t salt,
                                                          float *__restrict__ part) {
  extern __shared__ float red[];
  const BnGeom g = bn_geom(C);
  const uint32_t key = drop_key(seed, salt);
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < R ? r0 + rpb : R;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.active) {
    const int c = g.cg * 4;
    float mu[4], rs[4], ga[4], be[4];
    load4(mean + c, mu);
    load4(rstd + c, rs);
    load4(gamma + c, ga);
    load4(beta + c, be);
    for (int64_t r = r0 + g.rsub; r < r1; r += g.RPI) {
      float dp[4], zh[4];
      bn_dpre(dy, z, r, C, c, mu, rs, ga, be, use_tanh, key, thr, scale, dp, zh);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s1[q] += dp[q];
        s2[q] += dp[q] * zh[q];
      }
    }
  }
  bn_row_reduce(red, g, C, s1);
  bn_row_reduce(red, g, C, s2);
  if (g.active && g.rsub == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float *p = part + ((int64_t)blockIdx.x * C + g.cg * 4 + q) * 2;
      p[0] = s1[q];
      p[1] = s2[q];
    }
}

// dbeta = sum dpre, dgamma = sum dpre * zhat (in block order); sums kept for pass 2 in sums[2][C]
__global__ __launch_bounds__(256) void bn_bwd_finish_kernel(const float *__restrict__ part, int blocks, int C,
                                                            float *dgamma, float *dbeta, int accumulate,
                                                            float *__restrict__ sums) {
  const int64_t col = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);  // c * 2 + j
  const float v = parts_col_sum(part, blocks, 2LL * C, col);
  if (threadIdx.x >= 64 || col >= 2LL * C) return;
  const int c = (int)(col >> 1);
  if ((col & 1) == 0) {  // sum dpre
    sums[c] = v;
    dbeta[c] = accumulate ? dbeta[c] + v : v;
  } else {  // sum dpre * zhat
    sums[C + c] = v;
    dgamma[c] = accumulate ? dgamma[c] + v : v;
  }
}

// dz = gamma * rstd * (dpre - sum(dpre)/N - zhat * sum(dpre * zhat)/N) -> bf16
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float *__restrict__ dy, const float *__restrict__ z,
                                                           int64_t R, int C, const float *__restrict__ mean,
                                                           const float *__restrict__ rstd,
                                                           const float *__restrict__ gamma,
                                                           const float *__restrict__ beta, int use_tanh, uint32_t thr,
                                                           float scale, const int64_t *seed, uint32_t salt,
                                                           const float *__restrict__ sums, bf16 *__restrict__ dz) {
  const uint32_t key = drop_key(seed, salt);
  const float invn = 1.0f / (float)R;
  const int64_t n4 = R * (C >> 2);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / (C >> 2);
    const int c = (int)(i - row * (C >> 2)) * 4;
    float mu[4], rs[4], ga[4], be[4], s1[4], s2[4], dp[4], zh[4], o[4];
    load4(mean + c, mu);
    load4(rstd + c, rs);
    load4(gamma + c, ga);
    load4(beta + c, be);
    load4(sums + c, s1);
    load4(sums + C + c, s2);
    bn_dpre(dy, z, row, C, c, mu, rs, ga, be, use_tanh, key, thr, scale, dp, zh);
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = ga[q] * rs[q] * (dp[q] - s1[q] * invn - zh[q] * s2[q] * invn);
    store4(dz + row * C + c, o);
  }
}

int bn_blocks(int64_t R, int *rpb) {
  int nb = (int)(R < kBnBlocks ? (R > 0 ? R : 1) : kBnBlocks);
  *rpb = (int)((R + nb - 1) / nb);
  return nb;
}

unsigned bn_grid(int64_t R, int C) {
  const int64_t n = (R * (C >> 2) + 255) / 256;
  return (unsigned)(n < 1 ? 1 : (n > 4096 ? 4096 : n));
}

}  // namespace

extern "C" int64_t fs2_bn_train_ws_bytes(int C) { return (int64_t)kBnBlocks * C * 3 * (int64_t)sizeof(float) + 2LL * C * 4; }

extern "C" int fs2_bn_train_fwd(const float *z, int64_t R, int C, const float *gamma, const float *beta, float eps,
                                float momentum, float *running_mean, float *running_var, int use_tanh, float p_drop,
                                const int64_t *seed, int salt, const float *residual, void *y_bf, float *y_f32,
                                float *mean, float *rstd, float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (z == nullptr || gamma == nullptr || beta == nullptr || mean == nullptr || rstd == nullptr || ws == nullptr ||
      (y_bf == nullptr && y_f32 == nullptr))
    return FS2_EINVAL;
  if (R <= 0 || C <= 0 || (C & 3) || C > 1024 || !(p_drop >= 0.0f && p_drop < 1.0f) ||
      (p_drop > 0.0f && seed == nullptr) || ((running_mean == nullptr) != (running_var == nullptr)))
    return FS2_EINVAL;
  if (ws_bytes < fs2_bn_train_ws_bytes(C)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  int rpb;
  const int nb = bn_blocks(R, &rpb);
  const size_t lds = (size_t)(256 / (C >> 2)) * C * sizeof(float);
  hipLaunchKernelGGL(bn_stats_part_kernel, dim3(nb), dim3(256), lds, s, z, R, C, rpb, ws);
  hipLaunchKernelGGL(bn_stats_finish_kernel, dim3((2 * C + 63) / 64), dim3(256), 0, s, z, R, ws, nb, C, eps, momentum,
                     running_mean, running_var, mean, rstd);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(bn_grid(R, C)), dim3(256), 0, s, z, R, C, mean, rstd, gamma, beta, use_tanh,
                     drop_threshold(p_drop), 1.0f / (1.0f - p_drop), seed, (uint32_t)salt, residual,
                     reinterpret_cast<bf16 *>(y_bf), y_f32);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_bn_train_bwd(const float *dy, const float *z, int64_t R, int C, const float *gamma,
                                const float *beta, const float *mean, const float *rstd, int use_tanh, float p_drop,
                                const int64_t *seed, int salt, void *dz, float *dgamma, float *dbeta, int accumulate,
                                float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dy == nullptr || z == nullptr || gamma == nullptr || beta == nullptr || mean == nullptr || rstd == nullptr ||
      dz == nullptr || dgamma == nullptr || dbeta == nullptr || ws == nullptr)
    return FS2_EINVAL;
  if (R <= 0 || C <= 0 || (C & 3) || C > 1024 || !(p_drop >= 0.0f && p_drop < 1.0f) ||
      (p_drop > 0.0f && seed == nullptr))
    return FS2_EINVAL;
  if (ws_bytes < fs2_bn_train_ws_bytes(C)) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  int rpb;
  const int nb = bn_blocks(R, &rpb);
  const size_t lds = (size_t)(256 / (C >> 2)) * C * sizeof(float);
  const uint32_t thr = drop_threshold(p_drop);
  const float scale = 1.0f / (1.0f - p_drop);
  float *sums = ws + (int64_t)kBnBlocks * C * 3;
  hipLaunchKernelGGL(bn_bwd_part_kernel, dim3(nb), dim3(256), lds, s, dy, z, R, C, rpb, mean, rstd, gamma, beta,
                     use_tanh, thr, scale, seed, (uint32_t)salt, ws);
  hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3((2 * C + 63) / 64), dim3(256), 0, s, ws, nb, C, dgamma, dbeta, accumulate,
                     sums);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(bn_grid(R, C)), dim3(256), 0, s, dy, z, R, C, mean, rstd, gamma, beta,
                     use_tanh, thr, scale, seed, (uint32_t)salt, sums, reinterpret_cast<bf16 *>(dz));
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// clip_grad_norm_ + Adam (torch.optim.Adam, fused / capturable semantics; train.py:93-95 via
// ScheduledOptim.step_and_update_lr) over the flat gradient buffer in two launches:
//   1. per-block sums of squares of the flat gradients (block 0 also advances every step counter);
//   2. every block re-adds the partials in the same order (deterministic total norm), coef =
//      min(1, max_norm / (norm + 1e-6)); per element g *= coef (written back, as clip_grad_norm_
//      leaves the clipped gradients), g += wd * p, m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2,
//      p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
// Parameters are separate tensors, their gradients contiguous in the flat buffer at desc.off.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kAdamNormBlocks = 1024;

__global__ __launch_bounds__(256) void adam_norm_kernel(const float *__restrict__ g, int64_t n,
                                                        const fs2_adam_param *__restrict__ d, int np,
                                                        float *__restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4 *>(g)[i];
    s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = g[(n4 << 2) + threadIdx.x];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < np; i += 256)
      if (d[i].step != nullptr) d[i].step[0] += 1.0f;
}

__global__ __launch_bounds__(256) void adam_kernel(float *__restrict__ g, int64_t n, const float *__restrict__ part,
                                                   const fs2_adam_param *__restrict__ d, int np, const float *lr_ptr,
                                                   float lr_val, float b1, float b2, float eps, float wd,
                                                   float max_norm) {
  __shared__ float red[4];
  __shared__ float coef_s;
  float coef = 1.0f;
  if (max_norm > 0.0f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < kAdamNormBlocks; i += 256) s += part[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
      coef_s = fminf(max_norm / (norm + 1e-6f), 1.0f);
    }
    __syncthreads();
    coef = coef_s;
  }
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_val;
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 3) / 4 * 4;
  const int64_t e0 = (int64_t)blockIdx.x * per, e1 = e0 + per < n ? e0 + per : n;
  if (e0 >= e1) return;
  // parameter holding e0: last desc with off <= e0 (binary search)
  int lo = 0, hi = np - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].off <= e0) lo = mid; else hi = mid - 1;
  }
  int pi = lo;
  int64_t pend = d[pi].off + d[pi].numel;
  float step_size = 0.f, bc2s = 1.f;
  auto param_consts = [&]() {
    const float t = d[pi].step != nullptr ? d[pi].step[0] : 1.0f;
    const float bc1 = 1.0f - powf(b1, t), bc2 = 1.0f - powf(b2, t);
    step_size = lr / bc1;
    bc2s = sqrtf(bc2);
  };
  param_consts();
  // 4 consecutive elements per thread: a group lies in one parameter (16-byte aligned starts) or
  // in the zero gap after it; whole groups use 16-byte accesses, a parameter's ragged end scalars
  auto upd = [&](float gr, float &pv, float &mv, float &vv) __attribute__((always_inline)) {
    if (wd != 0.0f) gr += wd * pv;
    mv = b1 * mv + (1.0f - b1) * gr;
    vv = b2 * vv + (1.0f - b2) * gr * gr;
    pv = pv - step_size * mv / (sqrtf(vv) / bc2s + eps);
  };
  for (int64_t e = e0 + 4 * threadIdx.x; e < e1; e += 1024) {
    if (e >= pend) {
      while (e >= d[pi].off + d[pi].numel && pi + 1 < np && e >= d[pi + 1].off) ++pi;
      pend = d[pi].off + d[pi].numel;
      param_consts();
    }
    if (e < d[pi].off || e >= pend) {  // the gap after a parameter (zeros, nothing to update)
      if (max_norm > 0.0f) *reinterpret_cast<float4 *>(g + e) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    const int64_t j = e - d[pi].off;
    float4 gv = *reinterpret_cast<const float4 *>(g + e);
    if (max_norm > 0.0f) {
      gv.x *= coef, gv.y *= coef, gv.z *= coef, gv.w *= coef;
      *reinterpret_cast<float4 *>(g + e) = gv;
    }
    float *pp = d[pi].p + j, *mp = d[pi].m + j, *vp = d[pi].v + j;
    if (j + 4 <= d[pi].numel) {
      float4 pv = *reinterpret_cast<const float4 *>(pp), mv = *reinterpret_cast<const float4 *>(mp),
             vv = *reinterpret_cast<const float4 *>(vp);
      upd(gv.x, pv.x, mv.x, vv.x);
      upd(gv.y, pv.y, mv.y, vv.y);
      upd(gv.z, pv.z, mv.z, vv.z);
      upd(gv.w, pv.w, mv.w, vv.w);
      *reinterpret_cast<float4 *>(pp) = pv;
      *reinterpret_cast<float4 *>(mp) = mv;
      *reinterpret_cast<float4 *>(vp) = vv;
    } else {
      const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
      for (int q = 0; q < 4 && j + q < d[pi].numel; ++q) upd(gs[q], pp[q], mp[q], vp[q]);
    }
  }
}

}  // namespace

extern "C" int64_t fs2_adam_ws_bytes(void) { return (int64_t)kAdamNormBlocks * (int64_t)sizeof(float); }

extern "C" int fs2_adam_flat(float *grads, int64_t n, const fs2_adam_param *params_dev, int np, const float *lr_dev,
                             float lr, float beta1, float beta2, float eps, float weight_decay, float max_norm,
                             float *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (grads == nullptr || params_dev == nullptr || np <= 0 || ws == nullptr || n < 0 || (n & 3) ||
      (reinterpret_cast<uintptr_t>(grads) & 15))
    return FS2_EINVAL;
  if (ws_bytes < fs2_adam_ws_bytes()) return FS2_EINVAL;
  if (n == 0) return FS2_OK;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(adam_norm_kernel, dim3(kAdamNormBlocks), dim3(256), 0, s, grads, n, params_dev, np, ws);
  int64_t blocks = (n + 4095) / 4096;
  blocks = blocks > 8192 ? 8192 : blocks;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, grads, n, ws, params_dev, np, lr_dev, lr,
                     beta1, beta2, eps, weight_decay, max_norm);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_ln_bwd_parts(int64_t R) {
  const int64_t b64 = (R + 3) / 4;
  return R <= 0 ? 1 : (int)(b64 < kLnBlocks ? b64 : kLnBlocks);
}

// ---------------------------------------------------------------------------------------------
// Deferred split-partial reductions of a backward pass in one launch (per <= 32 of them): the
// weight / bias / LayerNorm-parameter gradients of the fused training nodes are only read by the
// optimizer, so their finish passes are batched after the backward instead of one small launch
// each. Same fixed-order sums as the immediate finish kernels (parts_col_sum).
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kReduceLongS = 16;  // more partials than this: the 64-column, 4-wave path

// one thread = 4 consecutive columns (16-byte partial loads, the S splits summed in order): the
// partial buffers are large (up to 8 x 9.4 MB for the FFN w_1 gradient) and S small
__global__ __launch_bounds__(256) void reduce_batch_kernel(fs2_reduce_batch a) {
  int i = 0;
  for (int j = 1; j < a.n; ++j)
    if (a.d[j].blk0 <= (int64_t)blockIdx.x) i = j;
  const fs2_reduce_desc &d = a.d[i];
  if (d.kind == 1 && d.KS > 1) {
    // a wide-tap weight gradient: partials [S][KS][N][C] -> out[n][c][k]. The plain mapping below
    // scatters every store KS floats apart (36 B at KS = 9: a partial line per 4 bytes, read-modify-
    // write when accumulating); here a block owns (n, 256 channels): each thread sums its channel's
    // KS taps over the S splits (coalesced loads per tap, the same fixed split order), the block
    // transposes them through LDS and stores its 256 x KS contiguous outputs coalesced.
    __shared__ float tr[256 * 9];
    const int KS = d.KS, C = d.C, N = d.N;
    const int cb = (C + 255) / 256;
    const int64_t bl = (int64_t)blockIdx.x - d.blk0;
    const int n = (int)(bl / cb), c0 = (int)(bl - (int64_t)n * cb) * 256;
    const int cn = min(256, C - c0), t = threadIdx.x;
    const int which = n / d.split;
    float *base = which == 0 ? d.out0 : which == 1 ? d.out1 : d.out2;
    float *dst = base == nullptr ? nullptr : base + ((int64_t)(n - which * d.split) * C + c0) * KS;
    // accumulating: the outputs' old values are loaded first, beside the partials (a load-add-store
    // per output after the sums paid one more memory latency per store)
    float old[9];
    const int ne = cn * KS;
#pragma unroll
    for (int i = 0; i < 9; ++i) old[i] = (dst != nullptr && d.accumulate && t + 256 * i < ne) ? dst[t + 256 * i] : 0.f;
    if (t < cn) {
      // every (tap, split) load issued before the first add (a dependent loop paid one memory
      // latency per load: ~100 us per batched launch); S <= 8 for wide taps (wgrad_splits)
      const float *pp = d.part + (int64_t)n * C + c0 + t;
      const int64_t NC = (int64_t)N * C;
      float v[9][8];
#pragma unroll
      for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
          v[k][s2] = (k < KS && s2 < d.S) ? pp[(int64_t)s2 * d.M + k * NC] : 0.0f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (k < KS) {
          float acc = v[k][0];
#pragma unroll
          for (int s2 = 1; s2 < 8; ++s2)
            if (s2 < d.S) acc += v[k][s2];
          tr[t * KS + k] = acc;
        }
      }
    }
    __syncthreads();
    if (dst == nullptr) return;
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (t + 256 * i < ne) dst[t + 256 * i] = old[i] + tr[t + 256 * i];
    return;
  }
  // output column -> destination (kind 0: row split into up to 3 vectors; kind 2: a vector and one
  // scalar; kind 1: weight gradient partials [S][KS][N][C] -> out[n][c][k], rows split into parameters)
  auto where = [&](int64_t col) -> float * {
    float *base;
    int64_t off;
    if (d.kind == 0) {
      const int64_t which = col / d.split;
      base = which == 0 ? d.out0 : which == 1 ? d.out1 : d.out2;
      off = col - which * d.split;
    } else if (d.kind == 2) {  // m < split -> out0[m], m == split -> out1[0]
      if (col > d.split) return nullptr;
      base = col < d.split ? d.out0 : d.out1;
      off = col < d.split ? col : 0;
    } else {
      const int64_t NC = (int64_t)d.N * d.C;
      const int k = (int)(col / NC);
      const int64_t nc = col - (int64_t)k * NC;
      const int n = (int)(nc / d.C), which = n / d.split;
      base = which == 0 ? d.out0 : which == 1 ? d.out1 : d.out2;
      off = (nc - (int64_t)which * d.split * d.C) * d.KS + k;
    }
    return base == nullptr ? nullptr : base + off;  // null: an output not wanted (no conv bias behind a LN)
  };
  // accumulating outputs: their old values are loaded before the partial sums (one latency, overlapped)
  auto old_of = [&](float *p) { return (p != nullptr && d.accumulate) ? *p : 0.f; };
  if (d.S > kReduceLongS) {
    // many partials of a short vector (LayerNorm parameters: 256 partial blocks x 768): a block owns
    // 64 columns, wave g sums partials g, g + 4, ... in order with every load of a 32-group issued
    // before its adds, the 4 wave sums added in a fixed order through LDS (the per-column loop of the
    // path below paid S / 8 memory latencies in ONE block: the tail of every batched launch)
    __shared__ float red[4][64];
    const int rg = threadIdx.x >> 6, cl = threadIdx.x & 63;
    const int64_t col = ((int64_t)blockIdx.x - d.blk0) * 64 + cl;
    float *dst = (rg == 0 && col < d.M) ? where(col) : nullptr;
    const float o = old_of(dst);
    float acc = 0.f;
    if (col < d.M) {
      for (int k0 = rg; k0 < d.S; k0 += 4 * 32) {
        float v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = k0 + 4 * j < d.S ? d.part[(int64_t)(k0 + 4 * j) * d.M + col] : 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) acc += v[j];
      }
    }
    red[rg][cl] = acc;
    __syncthreads();
    if (dst != nullptr) *dst = o + ((red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]));
    return;
  }
  const int64_t col0 = (((int64_t)blockIdx.x - d.blk0) * 256 + threadIdx.x) * 4;
  if (col0 >= d.M) return;
  float *dst[4];
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    dst[q] = where(col0 + q);
    o[q] = old_of(dst[q]);
  }
  // the splits in groups of 8: all 8 loads of a group issued before its adds (one memory latency per
  // group, not per split), summed in split order
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k0 = 0; k0 < d.S; k0 += 8) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = k0 + j < d.S ? *reinterpret_cast<const float4 *>(d.part + (int64_t)(k0 + j) * d.M + col0)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (k0 + j >= d.S) break;
      if (k0 + j == 0) {
        acc = v[0];
      } else {
        acc.x += v[j].x;
        acc.y += v[j].y;
        acc.z += v[j].z;
        acc.w += v[j].w;
      }
    }
  }
  const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (dst[q] != nullptr) *dst[q] = o[q] + vals[q];
}

}  // namespace

extern "C" int fs2_reduce_batch_launch(fs2_reduce_batch *a, fs2_stream_t stream) {
  if (a == nullptr || a->n <= 0 || a->n > FS2_REDUCE_BATCH_MAX) return FS2_EINVAL;
  int64_t blk = 0;
  for (int i = 0; i < a->n; ++i) {
    fs2_reduce_desc &d = a->d[i];
    if (d.part == nullptr || d.S <= 0 || d.M <= 0 || (d.M & 3) || d.split <= 0 || (d.kind < 0 || d.kind > 2) ||
        (reinterpret_cast<uintptr_t>(d.part) & 15))
      return FS2_EINVAL;
    if (d.kind == 1 && (d.KS <= 0 || d.KS > 9 || d.N <= 0 || d.C <= 0 || (int64_t)d.KS * d.N * d.C != d.M))
      return FS2_EINVAL;
    if (d.kind == 1 && d.KS > 1 && d.S > 8) return FS2_EINVAL;  // the wide-tap path sums <= 8 splits
    d.blk0 = blk;
    blk += d.kind == 1 && d.KS > 1 ? (int64_t)d.N * ((d.C + 255) / 256)
           : d.S > kReduceLongS     ? (d.M + 63) / 64
                                    : (d.M + 1023) / 1024;
  }
  if (blk >= (1LL << 31)) return FS2_EUNSUPPORTED;
  hipLaunchKernelGGL(reduce_batch_kernel, dim3((unsigned)blk), dim3(256), 0, as_stream(stream), *a);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

// ---------------------------------------------------------------------------------------------
// Backward of the conditioning add (model/fastspeech2.py:101-110 in training):
//   x + speaker_emb(s)[b] + relu(W cat(emo_emb(e), aro_emb(a), val_emb(v))[b] + bias)
// dc[b] = sum_l dy[b, l] (the broadcast's gradient), dh = dc * (relu output > 0); then the
// speaker / emotion / arousal / valence table rows, W and bias. Two launches, every sum in a fixed
// order (the batch entries that share an id are added to its row in batch order): deterministic.
// ---------------------------------------------------------------------------------------------
namespace {

// launch 1: (64 channels, one utterance) per workgroup: wave g sums positions g, g + 4, ... in order,
// the 4 wave sums added in a fixed order; writes dc and dh ([B][D] each) into the workspace
__global__ __launch_bounds__(256) void cond_colsum_kernel(const float *__restrict__ dy, int L, int D,
                                                          const float *__restrict__ emo_out, float *__restrict__ dc,
                                                          float *__restrict__ dh) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6, b = blockIdx.y, n = blockIdx.x * 64 + c;
  float acc = 0.f;
  if (n < D) {
    const float *p = dy + (int64_t)b * L * D + n;
    for (int l = g; l < L; l += 4) acc += p[(int64_t)l * D];
  }
  red[g][c] = acc;
  __syncthreads();
  if (g == 0 && n < D) {
    const float s = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    dc[(int64_t)b * D + n] = s;
    if (emo_out != nullptr) dh[(int64_t)b * D + n] = emo_out[(int64_t)b * D + n] > 0.f ? s : 0.f;
  }
}

// launch 2: three kinds of workgroups, by block index (none waits on another):
//  A  [0, nA): 16 Linear input columns k each: de[b][k] = sum_n dh[b][n] W[n][k] for every utterance
//     (dh and the W columns staged in LDS), then those columns of the emotion / arousal / valence
//     tables: each row = old + its utterances' de in batch order;
//  B  [nA, nA + nB): 4 rows n of dW each: dW[n][k] (+)= sum_b dh[b][n] cat[b][k];
//  C  the rest: 64 output channels each: the bias (sum over the batch) and the speaker rows.
// (One workgroup per 64 columns doing all of it ran ~30k dependent instructions per wave on 16
// waves: 90-150 us. Every global load here is unconditional at a clamped address, issued in
// batches before its use.)
constexpr int kCondKA = 16;  // Linear input columns per A workgroup
constexpr int kCondNB = 4;   // dW rows per B workgroup

__global__ __launch_bounds__(256) void cond_param_kernel(fs2_cond_desc f, fs2_cond_grads gr, int B, int D, int nA,
                                                         int nB, const float *__restrict__ dcw,
                                                         const float *__restrict__ dhw) {
  extern __shared__ float sm[];
  const int dcat = dhw != nullptr ? f.d_emo + f.d_aro + f.d_val : 0;
  const int tid = threadIdx.x, blk = blockIdx.x;
  auto clampi = [](int64_t v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : (int)v); };
  // table column k -> (table, source, gradient, row width, column in the row)
  auto col = [&](int k, int &t, const float *&src, float *&dst, const int64_t *&ids, int &nrow, int &dd, int &kk) {
    if (k >= f.d_emo + f.d_aro)
      t = 2, src = f.val_table, dst = gr.d_val_table, ids = f.valences, nrow = f.n_val, dd = f.d_val, kk = k - f.d_emo - f.d_aro;
    else if (k >= f.d_emo)
      t = 1, src = f.aro_table, dst = gr.d_aro_table, ids = f.arousals, nrow = f.n_aro, dd = f.d_aro, kk = k - f.d_emo;
    else
      t = 0, src = f.emo_table, dst = gr.d_emo_table, ids = f.emotions, nrow = f.n_emo, dd = f.d_emo, kk = k;
  };
  if (blk < nA) {
    // ---- A: de and the three tables' columns [k0, k0 + 16)
    float *dh = sm;                 // [B][D]
    float *ws = dh + B * D;         // [D][16] W columns
    float *de = ws + D * kCondKA;   // [B][16]
    float *ov = de + B * kCondKA;   // [B][16] old row values / running row sums
    int *idl = reinterpret_cast<int *>(ov + B * kCondKA);  // [3][B] rows, [3][B] reps
    const int k0 = blk * kCondKA;
    for (int i0 = tid; i0 < B * D; i0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = dhw[i0 + 256 * u < B * D ? i0 + 256 * u : B * D - 1];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + 256 * u < B * D) dh[i0 + 256 * u] = v[u];
    }
    for (int i0 = tid; i0 < D * kCondKA; i0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 256 * u < D * kCondKA ? i0 + 256 * u : D * kCondKA - 1;
        const int n = i / kCondKA, kc = k0 + (i - n * kCondKA);
        v[u] = f.lin_w[(int64_t)n * dcat + (kc < dcat ? kc : dcat - 1)];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + 256 * u < D * kCondKA) ws[i0 + 256 * u] = v[u];
    }
    for (int i = tid; i < 3 * B; i += 256) {
      const int t = i / B, b = i - t * B;
      idl[i] = t == 0 ? clampi(f.emotions[b], f.n_emo) : t == 1 ? clampi(f.arousals[b], f.n_aro)
                                                                 : clampi(f.valences[b], f.n_val);
    }
    __syncthreads();
    for (int i = tid; i < 3 * B; i += 256) {  // rep: the first utterance sharing the row
      const int t = i / B, b = i - t * B, r = idl[i];
      int f0 = b;
      for (int b2 = 0; b2 < b; ++b2)
        if (idl[t * B + b2] == r) {
          f0 = b2;
          break;
        }
      idl[3 * B + i] = f0;
    }
    // de: thread (column kc, utterance b = bb, bb + 16, ...), n in order
    const int kc = tid & (kCondKA - 1), bb = tid / kCondKA;
    for (int b = bb; b < B; b += 256 / kCondKA) {
      float a0 = 0.f, a1 = 0.f;  // two chains (even / odd n), added at the end
      const float *dr = dh + b * D;
      int n = 0;
      for (; n + 1 < D; n += 2) {
        a0 = fmaf(dr[n], ws[n * kCondKA + kc], a0);
        a1 = fmaf(dr[n + 1], ws[(n + 1) * kCondKA + kc], a1);
      }
      if (n < D) a0 = fmaf(dr[n], ws[n * kCondKA + kc], a0);
      de[b * kCondKA + kc] = a0 + a1;
    }
    // old values of every (utterance, column) row entry (only the reps' are used)
    for (int i = tid; i < B * kCondKA; i += 256) {
      const int b = i / kCondKA, k = k0 + (i - b * kCondKA);
      int t, nrow, dd, kk;
      const float *src;
      float *dst;
      const int64_t *ids;
      col(k < dcat ? k : dcat - 1, t, src, dst, ids, nrow, dd, kk);
      ov[i] = dst != nullptr ? dst[(int64_t)idl[t * B + b] * dd + kk] : 0.f;
    }
    __syncthreads();
    if (tid < kCondKA && k0 + tid < dcat) {
      const int k = k0 + tid;
      int t, nrow, dd, kk;
      const float *src;
      float *dst;
      const int64_t *ids;
      col(k, t, src, dst, ids, nrow, dd, kk);
      if (dst != nullptr) {
        for (int b = 0; b < B; ++b) ov[idl[3 * B + t * B + b] * kCondKA + tid] += de[b * kCondKA + tid];
        for (int b = 0; b < B; ++b)
          if (idl[3 * B + t * B + b] == b) dst[(int64_t)idl[t * B + b] * dd + kk] = ov[b * kCondKA + tid];
      }
    }
    return;
  }
  if (blk < nA + nB) {
    // ---- B: dW rows [n0, n0 + 4), every column k (the batch's cat column gathered per thread)
    if (gr.d_lin_w == nullptr) return;
    const int n0 = (blk - nA) * kCondNB;
    float *dhr = sm;  // [B][4] this workgroup's dh rows
    for (int i = tid; i < B * kCondNB; i += 256) {
      const int b = i / kCondNB, r = i - b * kCondNB;
      dhr[i] = dhw[(int64_t)b * D + (n0 + r < D ? n0 + r : D - 1)];
    }
    __syncthreads();
    for (int k = tid; k < dcat; k += 256) {
      int t, nrow, dd, kk;
      const float *src;
      float *dst;
      const int64_t *ids;
      col(k, t, src, dst, ids, nrow, dd, kk);
      float od[kCondNB], acc[kCondNB];
#pragma unroll
      for (int r = 0; r < kCondNB; ++r) {
        od[r] = gr.d_lin_w[(int64_t)(n0 + r < D ? n0 + r : D - 1) * dcat + k];
        acc[r] = 0.f;
      }
      for (int b0 = 0; b0 < B; b0 += 8) {
        float cv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int b = b0 + u < B ? b0 + u : B - 1;
          cv[u] = src[(int64_t)clampi(ids[b], nrow) * dd + kk];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (b0 + u >= B) break;
#pragma unroll
          for (int r = 0; r < kCondNB; ++r) acc[r] = fmaf(dhr[(b0 + u) * kCondNB + r], cv[u], acc[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < kCondNB; ++r)
        if (n0 + r < D) gr.d_lin_w[(int64_t)(n0 + r) * dcat + k] = od[r] + acc[r];
    }
    return;
  }
  // ---- C: output channels [n0, n0 + 64): bias and speaker rows
  const int n0 = (blk - nA - nB) * 64, c = tid & 63, g = tid >> 6;
  const int n = n0 + c, nc = n < D ? n : D - 1;
  float *dcb = sm;              // [B][64]
  float *ov = dcb + B * 64;     // [B][64]
  int *idl = reinterpret_cast<int *>(ov + B * 64);  // [B] rows, [B] reps
  const bool spk = f.speaker_table != nullptr && gr.d_speaker_table != nullptr;
  for (int b = tid; b < B; b += 256) idl[b] = spk ? clampi(f.speakers[b], f.n_speaker) : 0;
  __syncthreads();
  for (int b = tid; b < B; b += 256) {
    int f0 = b;
    for (int b2 = 0; b2 < b; ++b2)
      if (idl[b2] == idl[b]) {
        f0 = b2;
        break;
      }
    idl[B + b] = f0;
  }
  for (int b0 = g; b0 < B; b0 += 4 * 8) {
    float v[8], o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = b0 + 4 * u < B ? b0 + 4 * u : B - 1;
      v[u] = dcw[(int64_t)b * D + nc];
      o[u] = spk ? gr.d_speaker_table[(int64_t)idl[b] * D + nc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + 4 * u < B) dcb[(b0 + 4 * u) * 64 + c] = v[u], ov[(b0 + 4 * u) * 64 + c] = o[u];
  }
  float bs = 0.f;
  if (g == 0 && dcat && gr.d_lin_b != nullptr) {
    const float old = gr.d_lin_b[nc];
    for (int b0 = 0; b0 < B; b0 += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = dhw[(int64_t)(b0 + j < B ? b0 + j : B - 1) * D + nc];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (b0 + j < B) bs += v[j];
    }
    bs += old;
  }
  __syncthreads();
  if (g == 0 && n < D) {
    if (dcat && gr.d_lin_b != nullptr) gr.d_lin_b[n] = bs;
    if (spk) {
      for (int b = 0; b < B; ++b) ov[idl[B + b] * 64 + c] += dcb[b * 64 + c];
      for (int b = 0; b < B; ++b)
        if (idl[B + b] == b) gr.d_speaker_table[(int64_t)idl[b] * D + n] = ov[b * 64 + c];
    }
  }
}

}  // namespace

static size_t fs2_cond_bwd_smem(int B, int D, bool emo) {  // cond_param_kernel's LDS (the largest role)
  const size_t a = emo ? ((size_t)B * D + (size_t)D * kCondKA + 2 * (size_t)B * kCondKA) * sizeof(float) +
                             6 * (size_t)B * sizeof(int)
                       : 0;
  const size_t c = 2 * (size_t)B * 64 * sizeof(float) + 2 * (size_t)B * sizeof(int);
  return a > c ? a : c;
}

extern "C" int64_t fs2_cond_bwd_ws_bytes(int B, int D) {
  return B <= 0 || D <= 0 ? 0 : 2 * (int64_t)B * D * (int64_t)sizeof(float);
}

extern "C" int fs2_cond_bwd(const float *dy, int B, int L, int D, const fs2_cond_desc *fwd, const fs2_cond_grads *grads,
                            void *ws, int64_t ws_bytes, fs2_stream_t stream) {
  if (dy == nullptr || fwd == nullptr || grads == nullptr || ws == nullptr || B < 0 || L < 0 || D <= 0)
    return FS2_EINVAL;
  const fs2_cond_desc &f = *fwd;
  if (f.speaker_table != nullptr && (f.speakers == nullptr || f.n_speaker <= 0)) return FS2_EINVAL;
  if (f.emo_table != nullptr &&
      (f.emotions == nullptr || f.arousals == nullptr || f.valences == nullptr || f.aro_table == nullptr ||
       f.val_table == nullptr || f.lin_w == nullptr || f.emo_out == nullptr || f.n_emo <= 0 || f.n_aro <= 0 ||
       f.n_val <= 0 || f.d_emo <= 0 || f.d_aro <= 0 || f.d_val <= 0))
    return FS2_EINVAL;
  if (ws_bytes < fs2_cond_bwd_ws_bytes(B, D)) return FS2_EINVAL;
  if (B == 0 || L == 0 || (f.speaker_table == nullptr && f.emo_table == nullptr)) return FS2_OK;
  const size_t smem = fs2_cond_bwd_smem(B, D, f.emo_table != nullptr);
  if (B > 64 || smem > 65536) return FS2_EUNSUPPORTED;
  hipStream_t s = as_stream(stream);
  float *dc = static_cast<float *>(ws), *dh = dc + (int64_t)B * D;
  hipLaunchKernelGGL(cond_colsum_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)B), dim3(256), 0, s, dy, L, D,
                     f.emo_table != nullptr ? f.emo_out : nullptr, dc, dh);
  const int dcat = f.emo_table != nullptr ? f.d_emo + f.d_aro + f.d_val : 0;
  const int nA = (dcat + kCondKA - 1) / kCondKA, nB = dcat > 0 ? (D + kCondNB - 1) / kCondNB : 0;
  const int nC = (D + 63) / 64;
  hipLaunchKernelGGL(cond_param_kernel, dim3((unsigned)(nA + nB + nC)), dim3(256), smem, s, f, *grads, B, D, nA, nB,
                     dc, f.emo_table != nullptr ? dh : nullptr);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
