// The per-utterance conditioning vectors (model/fastspeech2.py:101-110), shared by fs2_cond_vectors
// (misc.hip) and the first encoder block's launch (enc_block.hip runs it on extra workgroups).
#pragma once
#include "fs2_common.h"

struct CondArgs {
  const int64_t *speakers;
  const float *spk_table;
  int n_spk;
  const int64_t *emotions;
  const float *emo_table;
  int n_emo, d_emo;
  const int64_t *arousals;
  const float *aro_table;
  int n_aro, d_aro;
  const int64_t *valences;
  const float *val_table;
  int n_val, d_val;
  const float *lin_w, *lin_b;
  int B, D;
  float *spk_out, *emo_out;
};

__device__ __forceinline__ int64_t cond_clampi(int64_t v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }

// Tile (channel block bx of 64, utterance block by of kCondU): the speaker rows are copied; the
// emotion Linear splits each channel's dot product over 4 waves (a quarter of k each, 16-byte
// weight loads), every weight read serving kCondU utterances, then sums the 4 partials in LDS.
// (One workgroup per utterance re-read the whole 256 KB weight 64 times: 13.5 us at cfg2.)
// Threads tid < 256 work; every thread of the workgroup must call it (it holds two barriers).
// sm: kCondU * (dc + 256) floats of LDS.
constexpr int kCondU = 8;

__device__ __forceinline__ void cond_tile(const CondArgs &a, int bx, int by, int tid, float *sm) {
  const bool act = tid < 256;
  const int n0 = bx * 64, b0 = by * kCondU;
  if (a.spk_table != nullptr && act) {
    for (int i = tid; i < kCondU * 64; i += 256) {
      const int b = b0 + (i >> 6), n = n0 + (i & 63);
      if (b < a.B && n < a.D) a.spk_out[(int64_t)b * a.D + n] = a.spk_table[cond_clampi(a.speakers[b], a.n_spk) * a.D + n];
    }
  }
  if (a.emo_table == nullptr) return;  // uniform over the workgroup
  const int dc = a.d_emo + a.d_aro + a.d_val;
  float *cat = sm;                   // [kCondU][dc]
  float *red = sm + kCondU * dc;     // [kCondU][4][64]
  if (act) {
    for (int i = tid; i < kCondU * dc; i += 256) {
      const int u = i / dc, k = i - u * dc, b = b0 + u;
      float x = 0.f;
      if (b < a.B) {
        if (k < a.d_emo)
          x = a.emo_table[cond_clampi(a.emotions[b], a.n_emo) * a.d_emo + k];
        else if (k < a.d_emo + a.d_aro)
          x = a.aro_table[cond_clampi(a.arousals[b], a.n_aro) * a.d_aro + (k - a.d_emo)];
        else
          x = a.val_table[cond_clampi(a.valences[b], a.n_val) * a.d_val + (k - a.d_emo - a.d_aro)];
      }
      cat[i] = x;
    }
  }
  __syncthreads();
  if (act) {
    const int nl = tid & 63, kq = tid >> 6, n = n0 + nl;
    float acc[kCondU];
#pragma unroll
    for (int u = 0; u < kCondU; ++u) acc[u] = 0.f;
    if (n < a.D) {
      const float *wr = a.lin_w + (int64_t)n * dc;
      if ((dc & 15) == 0) {
        const int kper = dc >> 2, k0 = kq * kper;
#pragma unroll 16
        for (int k = k0; k < k0 + kper; k += 4) {
          const float4 wv = *reinterpret_cast<const float4 *>(wr + k);
#pragma unroll
          for (int u = 0; u < kCondU; ++u) {
            const float4 c = *reinterpret_cast<const float4 *>(cat + u * dc + k);
            acc[u] = fmaf(wv.x, c.x, fmaf(wv.y, c.y, fmaf(wv.z, c.z, fmaf(wv.w, c.w, acc[u]))));
          }
        }
      } else {
        const int kper = (dc + 3) >> 2, k0 = kq * kper, k1 = min(dc, k0 + kper);
        for (int k = k0; k < k1; ++k) {
          const float wv = wr[k];
#pragma unroll
          for (int u = 0; u < kCondU; ++u) acc[u] = fmaf(wv, cat[u * dc + k], acc[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kCondU; ++u) red[(u * 4 + kq) * 64 + nl] = acc[u];
  }
  __syncthreads();
  if (act) {
    for (int i = tid; i < kCondU * 64; i += 256) {
      const int u = i >> 6, c = i & 63, b = b0 + u, nn = n0 + c;
      if (b < a.B && nn < a.D) {
        const float *r = red + u * 256 + c;
        a.emo_out[(int64_t)b * a.D + nn] = fmaxf(((r[0] + r[64]) + (r[128] + r[192])) + a.lin_b[nn], 0.f);
      }
    }
  }
}
