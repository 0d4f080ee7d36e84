// Backward of the key-padding-masked self-attention (training, cfg3) on CDNA4 MFMA, bf16 or f32.
//
// Reference: autograd through transformer/Modules.py:14-25 (S = Q K^T / temperature,
// masked_fill(key pad, -inf), softmax(dim=2), O = P V) and the head split/merge of
// transformer/SubLayers.py:36-52. The reference (and round 1 here) materialises the [H*B, T, T]
// score / probability / gradient tensors; this is a two-kernel flash-style backward that never
// writes a T x T tensor:
//
//   attn_bwd_dq_kernel   one workgroup per (64 queries, head, sequence): pass 1 over the key tiles
//                        rebuilds the softmax statistics (row max, sum -> lse), pass 2 recomputes
//                        P = exp(S - lse), dP = dO V^T, dS = P (dP - D) with D = rowsum(dO * O),
//                        and accumulates dQ = dS K / temperature in registers; lse and D go to a
//                        small f32 workspace [rows, H] for the second kernel.
//   attn_bwd_dkv_kernel  one workgroup per (64 keys, head, sequence), K and V rows in registers,
//                        loops over the query tiles: P^T, dS^T from K Q^T and V dO^T with the
//                        saved lse / D, dV += P^T dO, dK += dS^T Q / temperature.
//
// Both run the MFMA 16x16x32 bf16 or (exact f32) 16x16x4 f32 with the same fragment scheme as
// the forward's f32 kernel: a fragment is 16 bytes of consecutive k per lane (8 bf16 / 4 f32), a
// k-chunk is 4 lane groups of it (32 / 16 k); f32 issues 4 MFMAs per chunk with the same k
// permutation on both operands. Operands that an MFMA needs along the other axis (K, Q, dO for the
// gradient GEMMs) are staged transposed in LDS; C-layout results that feed the next MFMA as the A
// operand (dS, P^T) go through a wave-private LDS tile. Keys >= the sequence length get zero
// probability; every query row < T is computed (padded query rows attend to the valid keys, as
// in the reference); a zero-length sequence yields zero gradients.
#include "fs2_common.h"

namespace {

constexpr int DK = 128;

template <int CT>
struct BT;
template <>
struct BT<FS2_BF16> {
  using T = bf16;
  using Frag = bf16x8;
  static constexpr int KE = 8;  // elements per lane per fragment
};
template <>
struct BT<FS2_F32> {
  using T = float;
  using Frag = f32x4;
  static constexpr int KE = 4;
};

template <int CT>
__device__ __forceinline__ f32x4 mma(const typename BT<CT>::Frag &a, const typename BT<CT>::Frag &b, f32x4 c) {
  if constexpr (CT == FS2_BF16) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
    return c;
  }
}

template <int CT>
__device__ __forceinline__ typename BT<CT>::Frag ld_frag(const char *p) {
  return *reinterpret_cast<const typename BT<CT>::Frag *>(p);
}

template <typename TE>
__device__ __forceinline__ float to_f(TE v) {
  return (float)v;
}

// Sequence rows of (b): padded layout rows b*T .. (all T query rows exist, keys < len valid) or
// packed rows cu[b] .. cu[b+1]-1 (T = len).
__device__ __forceinline__ void seq_rows(const int64_t *lens, const int32_t *cu, int b, int &T, int &len,
                                         int64_t &row0) {
  if (cu != nullptr) {
    row0 = cu[b];
    len = cu[b + 1] - cu[b];
    T = len;
  } else {
    const int64_t l = lens[b];
    len = (int)(l < 0 ? 0 : (l > T ? T : l));
    row0 = (int64_t)b * T;
  }
}

// ------------------------------------------------------------------------------------------------
// dQ (+ lse, D).  4 waves x 16 queries.
template <int CT>
__global__ __launch_bounds__(256, 1) void attn_bwd_dq_kernel(const typename BT<CT>::T *__restrict__ qkv, int64_t qs,
                                                             const typename BT<CT>::T *__restrict__ o, int64_t os,
                                                             const float *__restrict__ dout, int64_t ds,
                                                             const int64_t *__restrict__ lens,
                                                             const int32_t *__restrict__ cu, int T, int H,
                                                             float scale_log2, float inv_temp,
                                                             float *__restrict__ dqkv, int64_t dqs,
                                                             float *__restrict__ lse_ws, float *__restrict__ d_ws,
                                                             const float *__restrict__ lse_in) {
  using TE = typename BT<CT>::T;
  using Frag = typename BT<CT>::Frag;
  constexpr int ES = sizeof(TE), KE = BT<CT>::KE, CK = 4 * KE, NCH = DK / CK;
  constexpr int KT = 64;                      // keys per tile
  constexpr int RS = DK * ES + 16;            // row stride of K / V tiles (bytes, padded)
  constexpr int TS = KT * ES + 16;            // row stride of Kt / dS tiles
  __shared__ __attribute__((aligned(16))) char Ks[KT * RS];
  __shared__ __attribute__((aligned(16))) char Vs[KT * RS];
  __shared__ __attribute__((aligned(16))) char Kt[DK * TS];
  __shared__ __attribute__((aligned(16))) char Ds[4 * 16 * TS];
  __shared__ float Drow[4][16];

  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  int len;
  int64_t row0;
  seq_rows(lens, cu, b, T, len, row0);
  if (q0 >= T) return;
  const int qrow = q0 + 16 * w + li;  // A-operand row of this lane
  const bool q_ok = qrow < T;

  // Q and dO fragments (A operands: row = query, k = head dim), D = rowsum(dO * O) per query
  Frag qf[NCH], dof[NCH];
  float dpart = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int d = c * CK + g * KE;
    if (q_ok) {
      qf[c] = ld_frag<CT>(reinterpret_cast<const char *>(qkv + (row0 + qrow) * qs + h * DK + d));
      float dv[KE], ov[KE];
      const float *dp = dout + (row0 + qrow) * ds + h * DK + d;
      const TE *op = o + (row0 + qrow) * os + h * DK + d;
#pragma unroll
      for (int e = 0; e < KE; ++e) {
        dv[e] = dp[e];
        ov[e] = to_f(op[e]);
        dpart += dv[e] * ov[e];
        dof[c][e] = (TE)dv[e];
      }
    } else {
      qf[c] = Frag{};
      dof[c] = Frag{};
    }
  }
  dpart += __shfl_xor(dpart, 16, 64);
  dpart += __shfl_xor(dpart, 32, 64);  // every lane of column li: D of query row li
  if (g == 0) Drow[w][li] = dpart;
  __syncthreads();

  auto load_tile = [&](int k0, bool with_v) {
    __syncthreads();
    constexpr int CPR = DK * ES / 16;  // 16-byte chunks per row
    for (int e = tid; e < KT * CPR; e += 256) {
      const int r = e / CPR, c = e % CPR;
      const int key = k0 + r;
      uint4 kv = make_uint4(0u, 0u, 0u, 0u), vv = kv;
      if (key < len) {
        kv = *reinterpret_cast<const uint4 *>(qkv + (row0 + key) * qs + (H + h) * DK + c * (16 / ES));
        if (with_v) vv = *reinterpret_cast<const uint4 *>(qkv + (row0 + key) * qs + (2 * H + h) * DK + c * (16 / ES));
      }
      *reinterpret_cast<uint4 *>(Ks + r * RS + c * 16) = kv;
      if (with_v) {
        *reinterpret_cast<uint4 *>(Vs + r * RS + c * 16) = vv;
        TE kt[16 / ES];
        __builtin_memcpy(kt, &kv, 16);
#pragma unroll
        for (int q = 0; q < 16 / ES; ++q) *reinterpret_cast<TE *>(Kt + (c * (16 / ES) + q) * TS + r * ES) = kt[q];
      }
    }
    __syncthreads();
  };
  // S (C layout: rows 4g+j of the wave's 16 queries, key column ni*16 + li), log2 domain, masked
  auto scores = [&](int k0, f32x4 (&s)[4]) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) s[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        s[ni] = mma<CT>(qf[c], ld_frag<CT>(Ks + (ni * 16 + li) * RS + (c * CK + g * KE) * ES), s[ni]);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[ni][j] = (k0 + ni * 16 + li < len) ? s[ni][j] * scale_log2 : -INFINITY;
  };

  const int ntiles = (len + KT - 1) / KT;
  // ---- pass 1: softmax statistics of the rows 4g+j (skipped when the forward saved them)
  float m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  for (int kt = 0; kt < (lse_in == nullptr ? ntiles : 0); ++kt) {
    load_tile(kt * KT, false);
    f32x4 s[4];
    scores(kt * KT, s);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mx = -INFINITY;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) mx = fmaxf(mx, s[ni][j]);
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mn = fmaxf(m[j], mx);
      float sum = 0.f;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) sum += exp2f(s[ni][j] - mn);
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      l[j] = l[j] * exp2f(m[j] - mn) + sum;
      m[j] = mn;
    }
  }
  float lse[4], Dj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lse[j] = l[j] > 0.f ? m[j] + __log2f(l[j]) : INFINITY;  // no valid key: P = 0
    if (lse_in != nullptr) {
      const int q = q0 + 16 * w + 4 * g + j;
      lse[j] = q < T ? lse_in[(row0 + q) * H + h] : INFINITY;
    }
    Dj[j] = Drow[w][4 * g + j];
  }
  // ---- pass 2: dQ
  f32x4 dq[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  char *Dw = Ds + w * 16 * TS;
  for (int kt = 0; kt < ntiles; ++kt) {
    load_tile(kt * KT, true);
    f32x4 s[4], dp[4];
    scores(kt * KT, s);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) dp[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        dp[ni] = mma<CT>(dof[c], ld_frag<CT>(Vs + (ni * 16 + li) * RS + (c * CK + g * KE) * ES), dp[ni]);
    // dS = P (dP - D) -> wave-private LDS [16 queries][64 keys] (the A operand of dQ += dS K)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = exp2f(s[ni][j] - lse[j]);
        *reinterpret_cast<TE *>(Dw + (4 * g + j) * TS + (ni * 16 + li) * ES) = (TE)(p * (dp[ni][j] - Dj[j]));
      }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < KT / CK; ++c) {
      const Frag a = ld_frag<CT>(Dw + li * TS + (c * CK + g * KE) * ES);
#pragma unroll
      for (int ni = 0; ni < DK / 16; ++ni)
        dq[ni] = mma<CT>(a, ld_frag<CT>(Kt + (ni * 16 + li) * TS + (c * CK + g * KE) * ES), dq[ni]);
    }
  }
  // ---- store dQ (C layout) and the statistics for the dK / dV kernel
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + 16 * w + 4 * g + j;
    if (q >= T) continue;
    float *dr = dqkv + (row0 + q) * dqs + h * DK + li;
#pragma unroll
    for (int ni = 0; ni < DK / 16; ++ni) dr[ni * 16] = dq[ni][j] * inv_temp;
    if (li == 0) {
      if (lse_in == nullptr) lse_ws[(row0 + q) * H + h] = lse[j];
      d_ws[(row0 + q) * H + h] = Dj[j];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dK, dV.  4 waves x 16 keys; QT queries per tile (64 bf16, 32 f32: LDS).
template <int CT>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkv_kernel(const typename BT<CT>::T *__restrict__ qkv, int64_t qs,
                                                              const float *__restrict__ dout, int64_t ds,
                                                              const int64_t *__restrict__ lens,
                                                              const int32_t *__restrict__ cu, int T, int H,
                                                              float scale_log2, float inv_temp,
                                                              float *__restrict__ dqkv, int64_t dqs,
                                                              const float *__restrict__ lse_ws,
                                                              const float *__restrict__ d_ws) {
  using TE = typename BT<CT>::T;
  using Frag = typename BT<CT>::Frag;
  constexpr int ES = sizeof(TE), KE = BT<CT>::KE, CK = 4 * KE, NCH = DK / CK;
  constexpr int QT = CT == FS2_BF16 ? 64 : 32;  // queries per tile
  constexpr int NQB = QT / 16;                   // 16-query column blocks
  constexpr int RS = DK * ES + 16;               // Q / dO row stride
  constexpr int TS = QT * ES + 16;               // Qt / dOt / P / dS row stride
  __shared__ __attribute__((aligned(16))) char Qs[QT * RS];
  __shared__ __attribute__((aligned(16))) char Os[QT * RS];  // dO (compute dtype)
  __shared__ __attribute__((aligned(16))) char Qt[DK * TS];
  __shared__ __attribute__((aligned(16))) char Ot[DK * TS];
  __shared__ __attribute__((aligned(16))) char Pw[4 * 16 * TS];
  __shared__ __attribute__((aligned(16))) char Sw[4 * 16 * TS];
  __shared__ float lq[QT], dq_[QT];

  const int b = blockIdx.z, h = blockIdx.y, k0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  int len;
  int64_t row0;
  seq_rows(lens, cu, b, T, len, row0);
  if (k0 >= T) return;
  const int krow = k0 + 16 * w + li;
  const bool k_ok = krow < len;
  Frag kf[NCH], vf[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int d = c * CK + g * KE;
    if (k_ok) {
      kf[c] = ld_frag<CT>(reinterpret_cast<const char *>(qkv + (row0 + krow) * qs + (H + h) * DK + d));
      vf[c] = ld_frag<CT>(reinterpret_cast<const char *>(qkv + (row0 + krow) * qs + (2 * H + h) * DK + d));
    } else {
      kf[c] = Frag{};
      vf[c] = Frag{};
    }
  }
  f32x4 dk[DK / 16], dv[DK / 16];
#pragma unroll
  for (int i = 0; i < DK / 16; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  char *Pm = Pw + w * 16 * TS;
  char *Sm = Sw + w * 16 * TS;
  const bool any_key = k0 < len;  // workgroup-uniform: keys past len only get zero gradients
  const int nqt = any_key ? (T + QT - 1) / QT : 0;
  for (int qt = 0; qt < nqt; ++qt) {
    const int q0 = qt * QT;
    __syncthreads();
    constexpr int CPR = DK * ES / 16;
    for (int e = tid; e < QT * CPR; e += 256) {
      const int r = e / CPR, c = e % CPR;
      const int q = q0 + r;
      uint4 qv = make_uint4(0u, 0u, 0u, 0u);
      TE ov[16 / ES];
      if (q < T) {
        qv = *reinterpret_cast<const uint4 *>(qkv + (row0 + q) * qs + h * DK + c * (16 / ES));
        const float *dp = dout + (row0 + q) * ds + h * DK + c * (16 / ES);
#pragma unroll
        for (int i = 0; i < 16 / ES; ++i) ov[i] = (TE)dp[i];
      } else {
#pragma unroll
        for (int i = 0; i < 16 / ES; ++i) ov[i] = (TE)0.f;
      }
      *reinterpret_cast<uint4 *>(Qs + r * RS + c * 16) = qv;
      __builtin_memcpy(Os + r * RS + c * 16, ov, 16);
      TE qe[16 / ES];
      __builtin_memcpy(qe, &qv, 16);
#pragma unroll
      for (int i = 0; i < 16 / ES; ++i) {
        *reinterpret_cast<TE *>(Qt + (c * (16 / ES) + i) * TS + r * ES) = qe[i];
        *reinterpret_cast<TE *>(Ot + (c * (16 / ES) + i) * TS + r * ES) = ov[i];
      }
    }
    for (int r = tid; r < QT; r += 256) {
      const int q = q0 + r;
      lq[r] = q < T ? lse_ws[(row0 + q) * H + h] : INFINITY;
      dq_[r] = q < T ? d_ws[(row0 + q) * H + h] : 0.f;
    }
    __syncthreads();
    // S^T = K Q^T and dP^T = V dO^T (C layout: rows = keys 4g+j, columns = queries nb*16 + li)
    f32x4 st[NQB], dpt[NQB];
#pragma unroll
    for (int nb = 0; nb < NQB; ++nb) {
      st[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dpt[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int nb = 0; nb < NQB; ++nb) {
        const int off = (nb * 16 + li) * RS + (c * CK + g * KE) * ES;
        st[nb] = mma<CT>(kf[c], ld_frag<CT>(Qs + off), st[nb]);
        dpt[nb] = mma<CT>(vf[c], ld_frag<CT>(Os + off), dpt[nb]);
      }
#pragma unroll
    for (int nb = 0; nb < NQB; ++nb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qc = nb * 16 + li;
        const bool ok = k0 + 16 * w + 4 * g + j < len;
        const float p = ok ? exp2f(st[nb][j] * scale_log2 - lq[qc]) : 0.f;
        *reinterpret_cast<TE *>(Pm + (4 * g + j) * TS + qc * ES) = (TE)p;
        *reinterpret_cast<TE *>(Sm + (4 * g + j) * TS + qc * ES) = (TE)(p * (dpt[nb][j] - dq_[qc]));
      }
    __syncthreads();
    // dV += P^T dO, dK += dS^T Q  (A from the wave's LDS tiles, B from the transposed tiles)
#pragma unroll
    for (int c = 0; c < QT / CK; ++c) {
      const Frag pa = ld_frag<CT>(Pm + li * TS + (c * CK + g * KE) * ES);
      const Frag sa = ld_frag<CT>(Sm + li * TS + (c * CK + g * KE) * ES);
#pragma unroll
      for (int ni = 0; ni < DK / 16; ++ni) {
        const int off = (ni * 16 + li) * TS + (c * CK + g * KE) * ES;
        dv[ni] = mma<CT>(pa, ld_frag<CT>(Ot + off), dv[ni]);
        dk[ni] = mma<CT>(sa, ld_frag<CT>(Qt + off), dk[ni]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int key = k0 + 16 * w + 4 * g + j;
    if (key >= T) continue;
    float *kr = dqkv + (row0 + key) * dqs + (H + h) * DK + li;
    float *vr = dqkv + (row0 + key) * dqs + (2 * H + h) * DK + li;
#pragma unroll
    for (int ni = 0; ni < DK / 16; ++ni) {
      kr[ni * 16] = dk[ni][j] * inv_temp;  // zero for keys >= len (no query attends to them)
      vr[ni * 16] = dv[ni][j];
    }
  }
}

template <int CT>
void launch_bwd(const void *qkv, int64_t qs, const void *o, int64_t os, const float *dout, int64_t ds,
                const int64_t *lens, const int32_t *cu, int B, int T, int H, float temperature, float *dqkv,
                int64_t dqs, float *ws, const float *lse_in, hipStream_t s) {
  using TE = typename BT<CT>::T;
  const float scale_log2 = 1.4426950408889634f / temperature, inv_temp = 1.0f / temperature;
  float *lse_ws = ws, *d_ws = ws + (int64_t)B * T * H;
  dim3 grid((T + 63) / 64, H, B);
  hipLaunchKernelGGL(attn_bwd_dq_kernel<CT>, grid, dim3(256), 0, s, reinterpret_cast<const TE *>(qkv), qs,
                     reinterpret_cast<const TE *>(o), os, dout, ds, lens, cu, T, H, scale_log2, inv_temp, dqkv, dqs,
                     lse_ws, d_ws, lse_in);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<CT>, grid, dim3(256), 0, s, reinterpret_cast<const TE *>(qkv), qs, dout, ds,
                     lens, cu, T, H, scale_log2, inv_temp, dqkv, dqs, lse_in != nullptr ? lse_in : lse_ws, d_ws);
}

}  // namespace

extern "C" int fs2_attention_bwd(const void *qkv, int dtype, int64_t qkv_row_stride, const void *out,
                                 int64_t out_row_stride, const float *dout, int64_t dout_row_stride,
                                 const int64_t *key_lens, int B, int T, int H, int dk, float temperature,
                                 float *dqkv, int64_t dqkv_row_stride, const int32_t *seq_cu, float *ws,
                                 int64_t ws_bytes, const float *lse, fs2_stream_t stream) {
  if (qkv == nullptr || out == nullptr || dout == nullptr || dqkv == nullptr || ws == nullptr) return FS2_EINVAL;
  if ((key_lens == nullptr) == (seq_cu == nullptr)) return FS2_EINVAL;
  if (B < 0 || T < 0 || H <= 0 || dk != DK || temperature <= 0.f) return FS2_EINVAL;
  if (qkv_row_stride < 3LL * H * dk || out_row_stride < (int64_t)H * dk || dout_row_stride < (int64_t)H * dk ||
      dqkv_row_stride < 3LL * H * dk)
    return FS2_EINVAL;
  const int ce = dtype == FS2_BF16 ? 8 : 4;
  if ((qkv_row_stride % ce) || (out_row_stride % ce) || (dout_row_stride % 4) || (dqkv_row_stride % 4))
    return FS2_EINVAL;
  if (ws_bytes < 2LL * B * T * H * (int64_t)sizeof(float)) return FS2_EINVAL;
  if (B == 0 || T == 0) return FS2_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == FS2_BF16)
    launch_bwd<FS2_BF16>(qkv, qkv_row_stride, out, out_row_stride, dout, dout_row_stride, key_lens, seq_cu, B, T, H,
                         temperature, dqkv, dqkv_row_stride, ws, lse, s);
  else if (dtype == FS2_F32)
    launch_bwd<FS2_F32>(qkv, qkv_row_stride, out, out_row_stride, dout, dout_row_stride, key_lens, seq_cu, B, T, H,
                        temperature, dqkv, dqkv_row_stride, ws, lse, s);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
