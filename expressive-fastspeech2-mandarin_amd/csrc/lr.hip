// LengthRegulator on CDNA4: per-sequence duration scan + per-frame gather (HBM-bound).
//
// Reference: model/modules.py:161-194 (LengthRegulator.LR / expand / forward) and the pad()
// it calls, utils/tools.py:360-378. The reference walks B*L_max phonemes in Python, calls
// .item() on each duration (one device->host sync each on a GPU), expands with
// vec.expand(max(int(d), 0)), concatenates and zero-pads/crops to max_len.
//
// Here: launch 1 (one workgroup per sequence) turns durations into frame counts
// max(trunc(d), 0), wavefront-scans them into an inclusive prefix sum `cum` and writes
// mel_len (the uncropped total). Launch 2 (B x ceil(T_out/32) workgroups) binary-searches
// each output frame's source phoneme in `cum` (first i with cum[i] > t) and streams the
// D-wide row with 16-byte vector loads/stores; frames at or past min(mel_len, T_out) are
// zero. An optional f32 position-encoding row is added on the way out (Decoder input,
// transformer/Models.py:158-160) so the expanded tensor is written to HBM exactly once.
#include <cstdlib>
#include <type_traits>

#include "fs2_common.h"

namespace {

constexpr int kScanThreads = 256;
constexpr int kLdsCum = 2048;  // cum rows up to this many phonemes are searched in LDS

__device__ __forceinline__ int64_t frames_of(const void *dur, int kind, float d_control, int64_t idx,
                                             float *d_rounded) {
  if (kind == FS2_DUR_I64) {
    int64_t d = reinterpret_cast<const int64_t *>(dur)[idx];
    return d > 0 ? d : 0;
  }
  float v = reinterpret_cast<const float *>(dur)[idx];
  if (kind == FS2_DUR_LOGPRED) {
    // torch.clamp(torch.round(torch.exp(log_d) - 1) * d_control, min=0)  (modules.py:132-135)
    float r = rintf(expf(v) - 1.0f) * d_control;
    r = r < 0.0f ? 0.0f : r;
    if (d_rounded) d_rounded[idx] = r;
    v = r;
  }
  // int(expand_size) truncates toward zero; max(., 0)                 (modules.py:186-187)
  if (!(v > 0.0f)) return 0;
  if (v >= 9.2e18f) return INT64_MAX / 4;
  return (int64_t)v;
}

__global__ __launch_bounds__(kScanThreads) void lr_durations_kernel(const void *dur, int kind, float d_control, int L,
                                                                    int32_t *cum, int64_t *mel_len, float *d_rounded) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int per = (L + kScanThreads - 1) / kScanThreads;
  const int i0 = min(tid * per, L), i1 = min(i0 + per, L);
  const int64_t base = (int64_t)b * L;

  int64_t local = 0;
  for (int i = i0; i < i1; ++i) local += frames_of(dur, kind, d_control, base + i, nullptr);

  // inclusive wave scan, then across the 4 waves through LDS
  int64_t incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  __shared__ int64_t wave_tot[kScanThreads / 64];
  if (lane == 63) wave_tot[wid] = incl;
  __syncthreads();
  int64_t prefix = 0;
  for (int w = 0; w < wid; ++w) prefix += wave_tot[w];
  int64_t run = prefix + incl - local;  // exclusive prefix of this thread's span

  for (int i = i0; i < i1; ++i) {
    run += frames_of(dur, kind, d_control, base + i, d_rounded);
    cum[base + i] = (int32_t)(run < 0x7fffffff ? run : 0x7fffffff);
  }
  if (tid == kScanThreads - 1) {
    int64_t total = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) total += wave_tot[w];
    mel_len[b] = total;
  }
}

// kRowsPerBlock output frames per workgroup. The utterance's `cum` row is staged in LDS with one
// coalesced load (rows longer than kLdsCum search global memory), so each frame's binary search
// (first i with cum[i] > t) costs LDS latency, not log2(L) dependent global round trips; then
// each thread keeps UNR independent 16-byte row pieces in flight (all loads issued before the
// stores).
template <typename TX, typename TO, bool HAS_PE, int ROWS, bool NT>
__global__ __launch_bounds__(256) void lr_expand_kernel(const TX *__restrict__ x, const int32_t *__restrict__ cum,
                                                        const int64_t *__restrict__ mel_len, int L, int D, int T_out,
                                                        const float *__restrict__ pe, TO *__restrict__ out,
                                                        int32_t *__restrict__ index_map,
                                                        const int32_t *__restrict__ out_cu) {
  constexpr int UNR = ROWS / 8;  // D = 256 bf16: 32 16-byte pieces per row, 256 threads
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * ROWS;
  const int tid = threadIdx.x;
  // packed output (out_cu != NULL): only frames t < out_cu[b+1] - out_cu[b] exist, at row out_cu[b] + t
  const int t_end = out_cu != nullptr ? min(T_out, out_cu[b + 1] - out_cu[b]) : T_out;
  if (t0 >= t_end && index_map == nullptr) return;
  __shared__ int src[ROWS];
  __shared__ int32_t scum[kLdsCum];
  const int64_t ml = mel_len[b];
  const int lim = (int)(ml < (int64_t)T_out ? ml : (int64_t)T_out);
  const int32_t *c = cum + (int64_t)b * L;
  const bool in_lds = L <= kLdsCum;
  if (in_lds)
    for (int i = tid; i < L; i += 256) scum[i] = c[i];
  __syncthreads();
  const int32_t *sc = in_lds ? scum : c;
  if (tid < ROWS) {
    const int t = t0 + tid;
    int s = -1;
    if (t < lim) {
      int lo = 0, hi = L - 1;  // first i with cum[i] > t (exists because t < mel_len)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sc[mid] > t) hi = mid; else lo = mid + 1;
      }
      s = lo;
    }
    src[tid] = s;
    if (index_map != nullptr && t < T_out) index_map[(int64_t)b * T_out + t] = s;
  }
  __syncthreads();
  if (out == nullptr) return;  // index-map-only call (the training gather reads the map)
  const int vpr = D >> 3;
  const int rows = min(ROWS, t_end - t0);
  if (rows <= 0) return;
  const int total = rows * vpr;
  const TX *xb = x + (int64_t)b * L * D;
  TO *ob = out + ((out_cu != nullptr ? (int64_t)out_cu[b] : (int64_t)b * T_out) + t0) * D;
  for (int base = tid; base < total; base += 256 * UNR) {
    float v[UNR][8];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = base + u * 256;
      const int r = e / vpr;
      const int col = (e - r * vpr) << 3;
      const int s = e < total ? src[r] : -1;
      if (s >= 0) {
        load8(xb + (int64_t)s * D + col, v[u]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[u][q] = 0.0f;
      }
      if constexpr (HAS_PE) {
        if (e < total) {
          float p[8];
          load8(pe + (int64_t)(t0 + r) * D + col, p);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[u][q] += p[q];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = base + u * 256;
      if (e < total) {
        if constexpr (NT && sizeof(TO) == 2) {  // streaming output: non-temporal 16-byte stores
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)v[u][q];
          __builtin_nontemporal_store(o, reinterpret_cast<bf16x8 *>(ob + (int64_t)e * 8));
        } else {
          store8(ob + (int64_t)e * 8, v[u]);
        }
      }
    }
  }
}

template <typename TX, typename TO, int ROWS, bool NT>
void launch_expand_v(const void *x, const int32_t *cum, const int64_t *mel_len, int B, int L, int D, int T_out,
                     const float *pe, void *out, int32_t *index_map, const int32_t *out_cu, hipStream_t s) {
  dim3 grid((T_out + ROWS - 1) / ROWS, B);
  if (pe != nullptr)
    hipLaunchKernelGGL((lr_expand_kernel<TX, TO, true, ROWS, NT>), grid, dim3(256), 0, s,
                       reinterpret_cast<const TX *>(x), cum, mel_len, L, D, T_out, pe, reinterpret_cast<TO *>(out),
                       index_map, out_cu);
  else
    hipLaunchKernelGGL((lr_expand_kernel<TX, TO, false, ROWS, NT>), grid, dim3(256), 0, s,
                       reinterpret_cast<const TX *>(x), cum, mel_len, L, D, T_out, pe, reinterpret_cast<TO *>(out),
                       index_map, out_cu);
}

// 32 rows per workgroup + non-temporal output stores. Measured against 64 rows and / or plain
// stores (same box, us per launch, cfg2 / cfg4 stress): 9.2 / 24.2 vs 9.3-9.5 / 26.1-33.4 -- cfg4
// moves 152 MB, so this form streams 6.3 TB/s (79 % of the 8 TB/s HBM peak).
template <typename TX, typename TO>
void launch_expand(const void *x, const int32_t *cum, const int64_t *mel_len, int B, int L, int D, int T_out,
                   const float *pe, void *out, int32_t *index_map, const int32_t *out_cu, hipStream_t s) {
  launch_expand_v<TX, TO, 32, true>(x, cum, mel_len, B, L, D, T_out, pe, out, index_map, out_cu, s);
}

// LengthRegulator backward (training, model/modules.py:161-194 through autograd): the gather's
// gradient is, per phoneme i of utterance b, the sum of dy over its contiguous frame range
// [cum[i-1], cum[i]) clipped to the T output frames (frames past T -- the max_len / decoder crop --
// carry no gradient). A segmented sum in frame order: deterministic, no atomics (torch's gather
// backward is a scatter-add with float atomics). 8 phonemes per workgroup, D/8 lanes per phoneme,
// 8 f32 columns per lane; dy [B, T, D] and dx [B, L, D] f32, contiguous.
__global__ __launch_bounds__(256) void lr_bwd_kernel(const float *__restrict__ dy, const int32_t *__restrict__ cum,
                                                     int L, int D, int T, float *__restrict__ dx) {
  constexpr int PH = 8;
  const int b = blockIdx.y, i0 = blockIdx.x * PH;
  const int vpr = D >> 3;
  const int32_t *c = cum + (int64_t)b * L;
  const float *db = dy + (int64_t)b * T * D;
  for (int e = threadIdx.x; e < PH * vpr; e += 256) {
    const int i = i0 + e / vpr;
    if (i >= L) break;
    const int col = (e - (i - i0) * vpr) << 3;
    const int t0 = i == 0 ? 0 : min(c[i - 1], T);
    const int t1 = min(c[i], T);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t = t0; t < t1; ++t) {
      float v[8];
      load8(db + (int64_t)t * D + col, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
    store8(dx + ((int64_t)b * L + i) * D + col, acc);
  }
}

// The whole LengthRegulator stage in ONE launch (round 4): each workgroup (32 frames of one
// utterance) (1) re-derives the utterance's cumulative frame counts in LDS -- from the durations
// (scan) or from a cum row computed before the free-running host read --, (2) the decoder's packed
// layout offset cu[b] = sum_{j<b} clamp(lens[j], 0, T) by a block reduction over the B lengths
// (B <= 4096: at most 16 loads per thread), (3) its frames' rowmap / row_pos entries and (4) the
// gather (+ PE) into the packed rows. The utterance's first workgroup also stores cum, mel_len,
// d_rounded and cu[b] (cu[B] by the last utterance). Replaces lr_durations + seq_layout +
// lr_expand (three dependent launches; cfg2 ~25 us with the gaps).
struct LrFusedArgs {
  const void *x;
  const void *dur;
  int dur_kind;
  float d_control;
  const int32_t *cum_in;
  const int64_t *mel_len_in;
  const int64_t *lens;  // layout lengths (the decoder's mel lengths)
  int B, L, D, T;
  const float *pe;
  void *out;
  int32_t *cum;
  int64_t *mel_len;
  float *d_rounded;
  int32_t *cu;
  int2 *row_pos;
  int32_t *rowmap;
  int store;  // bf16 frame stores: 0 non-temporal, 1 plain, 2 write-through (sc1); FS2_LR_STORE (A/B)
  // optional projection of the gathered frames (fs2_lr_fused_proj): proj_out[row] =
  // bf16(proj_src[b, src] + proj_pe[t]) over NP columns -- the decoder's first Q|K|V by linearity
  const float *proj_src;
  const float *proj_pe;
  int NP;
  bf16 *proj_out;
  // padded output (fs2_length_regulate, the reference's [B, T, D] contract, utils/tools.py:360-378):
  // row b*T + t for every t < T, zeros past min(mel_len, T); no packed layout is written
  int padded;
  int32_t *index_map;  // optional [B, T] source phoneme per frame (-1 past the expanded length)
};

template <typename TX, typename TO, bool HAS_PE, int ROWS>
__global__ __launch_bounds__(256) void lr_fused_kernel(LrFusedArgs a) {
  constexpr int UNR = ROWS / 8 < 8 ? ROWS / 8 : 8;  // 16-byte pieces in flight per thread
  const int b = blockIdx.y, t0 = blockIdx.x * ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int L = a.L, T = a.T, D = a.D;
  __shared__ int32_t scum[kLdsCum];
  __shared__ int src[ROWS];
  __shared__ int64_t wtot[4];
  __shared__ int32_t wcu[4];
  __shared__ int64_t s_ml;
  const bool first = blockIdx.x == 0;
  auto clen = [&](int j) {
    const int64_t l = a.lens[j];
    return (int32_t)(l < 0 ? 0 : (l > T ? T : l));
  };
  // the packed offset's loads are issued first, so their latency overlaps the scan's
  int32_t part = 0;
  if (!a.padded)
    for (int j = tid; j < b; j += 256) part += clen(j);

  // (2) cumulative frames of utterance b
  if (a.dur != nullptr) {
    const int per = (L + 255) / 256;
    const int i0 = min(tid * per, L), i1 = min(i0 + per, L);
    const int64_t base = (int64_t)b * L;
    int64_t local = 0;
    for (int i = i0; i < i1; ++i) local += frames_of(a.dur, a.dur_kind, a.d_control, base + i, nullptr);
    int64_t incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int64_t run = incl - local;
    for (int w = 0; w < wv; ++w) run += wtot[w];
    for (int i = i0; i < i1; ++i) {
      run += frames_of(a.dur, a.dur_kind, a.d_control, base + i, first ? a.d_rounded : nullptr);
      const int32_t c = (int32_t)(run < 0x7fffffff ? run : 0x7fffffff);
      scum[i] = c;
      if (first) a.cum[base + i] = c;
    }
    if (tid == 0) {
      const int64_t total = (wtot[0] + wtot[1]) + (wtot[2] + wtot[3]);
      s_ml = total;
      if (first) a.mel_len[b] = total;
    }
  } else {
    const int32_t *c = a.cum_in + (int64_t)b * L;
    for (int i = tid; i < L; i += 256) scum[i] = c[i];
    if (tid == 0) s_ml = a.mel_len_in[b];
  }

  // (1) packed offset of utterance b and its clamped length (padded: row b*T, all T rows written)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (lane == 0) wcu[wv] = part;
  __syncthreads();
  const int32_t cu_b = a.padded ? b * T : (wcu[0] + wcu[1]) + (wcu[2] + wcu[3]);
  const int32_t len_b = a.padded ? T : clen(b);
  if (first && tid == 0 && !a.padded) {
    a.cu[b] = cu_b;
    if (b == a.B - 1) a.cu[a.B] = cu_b + len_b;
  }

  // (3) source phoneme of each frame; the layout entries of this workgroup's frames
  const int64_t ml = s_ml;
  const int lim = (int)(ml < (int64_t)T ? ml : (int64_t)T);
  if (tid < ROWS) {
    const int t = t0 + tid;
    int sidx = -1;
    if (t < lim) {
      int lo = 0, hi = L - 1;  // first i with cum[i] > t (exists because t < mel_len)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (scum[mid] > t) hi = mid; else lo = mid + 1;
      }
      sidx = lo;
    }
    src[tid] = sidx;
    if (a.index_map != nullptr && t < T) a.index_map[(int64_t)b * T + t] = sidx;
    if (t < T && !a.padded) {
      if (a.rowmap != nullptr) a.rowmap[(int64_t)b * T + t] = t < len_b ? cu_b + t : -1;
      if (a.row_pos != nullptr && t < len_b) a.row_pos[cu_b + t] = make_int2(t, len_b);
    }
  }
  __syncthreads();

  // (4) gather (+ PE) of the frames t < len_b into packed rows cu_b + t
  const int rows = min(ROWS, min(T, (int)len_b) - t0);
  if (rows <= 0) return;
  const int vpr = D >> 3, total = rows * vpr;
  const TX *xb = reinterpret_cast<const TX *>(a.x) + (int64_t)b * L * D;
  TO *ob = reinterpret_cast<TO *>(a.out) + ((int64_t)cu_b + t0) * D;
  // x (+ PE) gathered by all threads, then (with the projection) the Q|K|V rows by waves 0-2
  const bool proj = a.proj_out != nullptr;
  auto gather = [&](auto UC, int me, int nthr) {
    constexpr int U = decltype(UC)::value;
    for (int base = me; base < total; base += nthr * U) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * nthr;
        const int r = e / vpr;
        const int col = (e - r * vpr) << 3;
        const int sidx = e < total ? src[r] : -1;
        if (sidx >= 0) {
          load8(xb + (int64_t)sidx * D + col, v[u]);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[u][q] = 0.0f;
        }
        if constexpr (HAS_PE) {
          if (e < total) {
            float pv[8];
            load8(a.pe + (int64_t)(t0 + r) * D + col, pv);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[u][q] += pv[q];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * nthr;
        if (e < total) {
          if constexpr (sizeof(TO) == 2) {
            bf16x8 o;
#pragma unroll
            for (int q = 0; q < 8; ++q) o[q] = (bf16)v[u][q];
            bf16x8 *dst = reinterpret_cast<bf16x8 *>(ob + (int64_t)e * 8);
            if (a.store == 0)
              __builtin_nontemporal_store(o, dst);
            else if (a.store == 1)
              *dst = o;
            else
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o),
                                                     __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 16, 0x00020000), 0u,
                                                     0, 16);
          } else {
            store8(ob + (int64_t)e * 8, v[u]);
          }
        }
      }
    }
  };
  gather(std::integral_constant<int, UNR>{}, tid, 256);
  // (5) the projection: (x[src] + pe[t]) W + b = (x W)[src] + (pe W + b)[t], both f32, one bf16
  // rounding at the end. Waves 0-2: thread t owns 8 columns (t % 96) of every other row (t / 96)
  // and walks 8 of its rows per round with all 32 loads in flight (the table rows from L2, shared
  // by the B utterances; the phoneme rows mostly from L1, one phoneme serving ~7 consecutive
  // frames); 16-byte stores. Graph-timed alone at cfg2 (r5p): 24.2 us against 10.9 without the
  // projection -- the 38 MB of Q|K|V rows at ~5.8 TB/s, ~90 MB of L2 reads, ~4 us of loop.
  if (proj && wv < 3) {
    constexpr int RB = 8;
    const int NP = a.NP, cg = NP >> 3;  // 8-column groups per row (96 at NP = 768)
    const float *tb = a.proj_pe + (int64_t)t0 * NP;
    const float *sb = a.proj_src + (int64_t)b * L * NP;
    bf16 *pb = a.proj_out + ((int64_t)cu_b + t0) * NP;
    const int lanes = 192 / cg * cg;  // threads in use: whole rows of column groups
    if (tid < lanes) {
      const int c = (tid % cg) * 8, r1 = tid / cg, rs = lanes / cg;
      for (int r0 = r1; r0 < rows; r0 += RB * rs) {
        float4 tv[RB][2], sv[RB][2];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
          const int r = min(r0 + u * rs, rows - 1);
          const int sidx = src[r];
          const float *tp = tb + (int64_t)r * NP + c;
          tv[u][0] = *reinterpret_cast<const float4 *>(tp);
          tv[u][1] = *reinterpret_cast<const float4 *>(tp + 4);
          if (sidx >= 0) {
            const float *sp = sb + (int64_t)sidx * NP + c;
            sv[u][0] = *reinterpret_cast<const float4 *>(sp);
            sv[u][1] = *reinterpret_cast<const float4 *>(sp + 4);
          } else {
            sv[u][0] = sv[u][1] = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
          const int r = r0 + u * rs;
          if (r < rows) {
            const bf16x8 o{(bf16)(tv[u][0].x + sv[u][0].x), (bf16)(tv[u][0].y + sv[u][0].y),
                           (bf16)(tv[u][0].z + sv[u][0].z), (bf16)(tv[u][0].w + sv[u][0].w),
                           (bf16)(tv[u][1].x + sv[u][1].x), (bf16)(tv[u][1].y + sv[u][1].y),
                           (bf16)(tv[u][1].z + sv[u][1].z), (bf16)(tv[u][1].w + sv[u][1].w)};
            __builtin_nontemporal_store(o, reinterpret_cast<bf16x8 *>(pb + (int64_t)r * NP + c));
          }
        }
      }
    }
  }
}

// get_mask_from_lengths (utils/tools.py:152-160): mask[b, t] = t >= lens[b]  (True = padding)
__global__ __launch_bounds__(256) void length_mask_kernel(const int64_t *__restrict__ lens, int width, int64_t n,
                                                          bool *__restrict__ mask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t b = i / width;
  mask[i] = (int64_t)(i - b * width) >= lens[b];
}

// Packed-sequence layout: cu[b] = sum_{j<b} clamp(lens[j], 0, T), cu[B] = total rows; one workgroup.
__global__ __launch_bounds__(256) void seq_cu_kernel(const int64_t *__restrict__ lens, int B, int T,
                                                     int32_t *__restrict__ cu) {
  __shared__ int32_t part[257];
  const int tid = threadIdx.x;
  const int per = (B + 255) / 256;
  const int i0 = min(tid * per, B), i1 = min(i0 + per, B);
  int32_t local = 0;
  for (int i = i0; i < i1; ++i) {
    const int64_t l = lens[i];
    local += (int32_t)(l < 0 ? 0 : (l > T ? T : l));
  }
  part[tid + 1] = local;
  if (tid == 0) part[0] = 0;
  __syncthreads();
  if (tid == 0)
    for (int i = 1; i <= 256; ++i) part[i] += part[i - 1];
  __syncthreads();
  int32_t run = part[tid];
  for (int i = i0; i < i1; ++i) {
    cu[i] = run;
    const int64_t l = lens[i];
    run += (int32_t)(l < 0 ? 0 : (l > T ? T : l));
  }
  if (tid == 255) cu[B] = part[256];
}

// Over the padded frame index i = b*T + t, with len = cu[b+1] - cu[b]:
//   rowmap[i] = t < len ? cu[b] + t : -1          (padded row -> packed row)
//   row_pos[cu[b] + t] = {t, len}  for t < len    (packed row -> position in its sequence)
__global__ __launch_bounds__(256) void seq_rows_kernel(const int32_t *__restrict__ cu, int B, int T,
                                                       int2 *__restrict__ row_pos, int32_t *__restrict__ rowmap) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * T) return;
  const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
  const int c = cu[b], len = cu[b + 1] - c;
  if (rowmap != nullptr) rowmap[i] = t < len ? c + t : -1;
  if (row_pos != nullptr && t < len) row_pos[c + t] = make_int2(t, len);
}

// The two launches above as one (B <= kSeqMaxB): every workgroup recomputes cu[0..B] in LDS
// (clamped lengths, wave shuffle scan; B = 64 costs nothing) and writes its 256 padded frames;
// workgroup 0 also stores cu. One tiny launch less per layout.
constexpr int kSeqMaxB = 4096;
__global__ __launch_bounds__(256) void seq_layout_kernel(const int64_t *__restrict__ lens, int B, int T,
                                                         int32_t *__restrict__ cu, int2 *__restrict__ row_pos,
                                                         int32_t *__restrict__ rowmap, int margin) {
  __shared__ int32_t scu[kSeqMaxB + 1];
  __shared__ int32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (B + 255) / 256;
  const int i0 = min(tid * per, B), i1 = min(i0 + per, B);
  // margin > 0 (the PostNet valid-region rows): len + margin frames, or all T when len + 2 margin > T
  auto clen = [&](int i) {
    int64_t l = lens[i];
    if (margin > 0) l = l + 2 * (int64_t)margin > T ? T : l + margin;
    return (int32_t)(l < 0 ? 0 : (l > T ? T : l));
  };
  int32_t local = 0;
  for (int i = i0; i < i1; ++i) local += clen(i);
  int32_t v = local;  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[wv] = v;
  __syncthreads();
  int32_t run = v - local;
  for (int w = 0; w < wv; ++w) run += wsum[w];
  for (int i = i0; i < i1; ++i) {
    scu[i] = run;
    run += clen(i);
  }
  if (tid == 0) scu[B] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  if (blockIdx.x == 0)
    for (int i = tid; i <= B; i += 256) cu[i] = scu[i];
  const int64_t i = (int64_t)blockIdx.x * 256 + tid;
  if (i >= (int64_t)B * T) return;
  const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
  const int c = scu[b], len = scu[b + 1] - c;
  if (rowmap != nullptr) rowmap[i] = t < len ? c + t : -1;
  if (row_pos != nullptr && t < len) row_pos[c + t] = make_int2(t, len);
}

// [max(len), sum(len), *bad] as int32 (lengths clamped to [0, 2^31 - 1]): the free-running
// path's one host read in one launch. One workgroup.
__global__ __launch_bounds__(256) void len_stats_kernel(const int64_t *__restrict__ lens, int B,
                                                        const int32_t *__restrict__ bad, int32_t *__restrict__ meta) {
  __shared__ int64_t smax[4], ssum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int64_t mx = 0, sm = 0;
  for (int i = tid; i < B; i += 256) {
    const int64_t l = lens[i] < 0 ? 0 : lens[i];
    mx = l > mx ? l : mx;
    sm += l;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(mx, o), b = __shfl_xor(sm, o);
    mx = a > mx ? a : mx;
    sm += b;
  }
  if (lane == 0) {
    smax[wv] = mx;
    ssum[wv] = sm;
  }
  __syncthreads();
  if (tid == 0) {
    int64_t m = 0, t = 0;
    for (int w = 0; w < 4; ++w) {
      m = smax[w] > m ? smax[w] : m;
      t += ssum[w];
    }
    meta[0] = (int32_t)(m < 0x7fffffff ? m : 0x7fffffff);
    meta[1] = (int32_t)(t < 0x7fffffff ? t : 0x7fffffff);
    meta[2] = bad != nullptr ? *bad : 0;
  }
}

}  // namespace

extern "C" int fs2_seq_layout_margin(const int64_t *lens, int B, int T, int margin, int32_t *cu, int32_t *row_pos,
                                     int32_t *rowmap, fs2_stream_t stream) {
  if (lens == nullptr || cu == nullptr || B < 0 || T < 0 || margin < 0 || B > kSeqMaxB ||
      (int64_t)B * T > 0x7fffff00LL)
    return FS2_EINVAL;
  const int64_t n = (int64_t)B * T;
  hipLaunchKernelGGL(seq_layout_kernel, dim3((unsigned)(n > 0 ? (n + 255) / 256 : 1)), dim3(256), 0, as_stream(stream),
                     lens, B, T, cu, reinterpret_cast<int2 *>(row_pos), rowmap, margin);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_seq_layout(const int64_t *lens, int B, int T, int32_t *cu, int32_t *row_pos, int32_t *rowmap,
                              fs2_stream_t stream) {
  if (lens == nullptr || cu == nullptr || B < 0 || T < 0 || (int64_t)B * T > 0x7fffff00LL) return FS2_EINVAL;
  hipStream_t s = as_stream(stream);
  if (B <= kSeqMaxB) return fs2_seq_layout_margin(lens, B, T, 0, cu, row_pos, rowmap, stream);
  hipLaunchKernelGGL(seq_cu_kernel, dim3(1), dim3(256), 0, s, lens, B, T, cu);
  FS2_CHECK_LAUNCH();
  if ((rowmap != nullptr || row_pos != nullptr) && (int64_t)B * T > 0) {
    hipLaunchKernelGGL(seq_rows_kernel, dim3((unsigned)(((int64_t)B * T + 255) / 256)), dim3(256), 0, s, cu, B, T,
                       reinterpret_cast<int2 *>(row_pos), rowmap);
    FS2_CHECK_LAUNCH();
  }
  return FS2_OK;
}

extern "C" int fs2_length_masks(const int64_t *lens, int B, int width, bool *mask, fs2_stream_t stream) {
  if (lens == nullptr || mask == nullptr || B < 0 || width < 0) return FS2_EINVAL;
  const int64_t n = (int64_t)B * width;
  if (n == 0) return FS2_OK;
  hipLaunchKernelGGL(length_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), lens, width,
                     n, mask);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_lr_durations(const void *dur, int dur_kind, float d_control, int B, int L, int32_t *cum,
                                int64_t *mel_len, float *d_rounded, fs2_stream_t stream) {
  if (dur == nullptr || cum == nullptr || mel_len == nullptr || B < 0 || L <= 0) return FS2_EINVAL;
  if (dur_kind < FS2_DUR_I64 || dur_kind > FS2_DUR_LOGPRED) return FS2_EINVAL;
  if (B == 0) return FS2_OK;
  hipLaunchKernelGGL(lr_durations_kernel, dim3(B), dim3(kScanThreads), 0, as_stream(stream), dur, dur_kind, d_control,
                     L, cum, mel_len, d_rounded);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_lr_expand(const void *x, int x_dtype, const int32_t *cum, const int64_t *mel_len, int B, int L,
                             int D, int T_out, const float *pe, void *out, int out_dtype, int32_t *index_map,
                             const int32_t *out_cu, fs2_stream_t stream) {
  // out may be NULL when index_map is given: only the source-index map is written
  if (x == nullptr || cum == nullptr || mel_len == nullptr || (out == nullptr && index_map == nullptr))
    return FS2_EINVAL;
  if (B < 0 || L <= 0 || D <= 0 || (D & 7) != 0 || T_out < 0) return FS2_EINVAL;
  if (B == 0 || T_out == 0) return FS2_OK;
  hipStream_t s = as_stream(stream);
  if (x_dtype == FS2_F32 && out_dtype == FS2_F32)
    launch_expand<float, float>(x, cum, mel_len, B, L, D, T_out, pe, out, index_map, out_cu, s);
  else if (x_dtype == FS2_BF16 && out_dtype == FS2_BF16)
    launch_expand<bf16, bf16>(x, cum, mel_len, B, L, D, T_out, pe, out, index_map, out_cu, s);
  else if (x_dtype == FS2_F32 && out_dtype == FS2_BF16)
    launch_expand<float, bf16>(x, cum, mel_len, B, L, D, T_out, pe, out, index_map, out_cu, s);
  else if (x_dtype == FS2_BF16 && out_dtype == FS2_F32)
    launch_expand<bf16, float>(x, cum, mel_len, B, L, D, T_out, pe, out, index_map, out_cu, s);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

static int lr_fused_launch(const LrFusedArgs &a, int x_dtype, int out_dtype, hipStream_t s);

// fs2_length_regulate's kernel: the padded contract alone, sized for HBM streaming. Each workgroup
// owns FR frames of one utterance and re-derives the utterance's scan (L <= 1024 durations: <= 4 per
// thread, cached in registers), but where lr_fused_kernel binary-searches every frame's source in an
// LDS cum row (log2 L dependent LDS reads), each phoneme here PAINTS its frame range
// [cum[i-1], cum[i]) clipped to the workgroup's frames into src[] -- one pass, no dependent chain;
// the first i with cum[i] > t is exactly the phoneme whose range holds t. Then the FR x D gather
// (+ PE) with 8 x 16-byte pieces in flight per thread and non-temporal stores. No projection or packed
// layout code is compiled in: the lean register file keeps ~4 workgroups per CU resident, so one
// workgroup's scan runs under the others' streams (lr_fused_kernel in the padded mode carried the
// projection's registers: 44 us at cfg4, 0.42 of HBM).
template <typename TX, typename TO, bool HAS_PE, int FR>
__global__ __launch_bounds__(256) void lr_pad_kernel(LrFusedArgs a) {
  constexpr int PER = 4;  // durations per thread (L <= 1024)
  constexpr int U = 8;    // 16-byte pieces in flight per thread
  const int b = blockIdx.y, t0 = blockIdx.x * FR;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int L = a.L, T = a.T, D = a.D;
  __shared__ int src[FR];
  __shared__ int64_t wtot[4];
  const bool first = blockIdx.x == 0;
  if (tid < FR) src[tid] = -1;
  const int per = (L + 255) >> 8;
  const int i0 = min(tid * per, L), i1 = min(i0 + per, L);
  const int64_t base = (int64_t)b * L;
  int64_t fr[PER];
  int64_t local = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    fr[k] = i0 + k < i1 ? frames_of(a.dur, a.dur_kind, a.d_control, base + i0 + k, first ? a.d_rounded : nullptr) : 0;
    local += fr[k];
  }
  int64_t incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wtot[wv] = incl;
  __syncthreads();
  int64_t run = incl - local;
  for (int w = 0; w < wv; ++w) run += wtot[w];
  const int64_t f0 = t0, f1 = min(t0 + FR, T);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (i0 + k < i1) {
      const int64_t s = run;
      run += fr[k];
      if (first) a.cum[base + i0 + k] = (int32_t)(run < 0x7fffffff ? run : 0x7fffffff);
      const int lo = (int)(s > f0 ? s : f0), hi = (int)(run < f1 ? run : f1);
      for (int t = lo; t < hi; ++t) src[t - t0] = i0 + k;
    }
  }
  if (first && tid == 0) a.mel_len[b] = (wtot[0] + wtot[1]) + (wtot[2] + wtot[3]);
  __syncthreads();
  if (a.index_map != nullptr && tid < FR && t0 + tid < T) a.index_map[(int64_t)b * T + t0 + tid] = src[tid];

  const int rows = min(FR, T - t0);
  const int vpr = D >> 3, total = rows * vpr;
  const TX *xb = reinterpret_cast<const TX *>(a.x) + base * D;
  TO *ob = reinterpret_cast<TO *>(a.out) + ((int64_t)b * T + t0) * D;
  for (int e0 = tid; e0 < total; e0 += 256 * U) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * 256;
      const int r = e / vpr, col = (e - r * vpr) << 3;
      const int s = e < total ? src[r] : -1;
      if (s >= 0) {
        load8(xb + (int64_t)s * D + col, v[u]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[u][q] = 0.0f;
      }
      if constexpr (HAS_PE) {
        if (e < total) {
          float pv[8];
          load8(a.pe + (int64_t)(t0 + r) * D + col, pv);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[u][q] += pv[q];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * 256;
      if (e < total) {
        if constexpr (sizeof(TO) == 2) {
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)v[u][q];
          __builtin_nontemporal_store(o, reinterpret_cast<bf16x8 *>(ob + (int64_t)e * 8));
        } else {
          store8(ob + (int64_t)e * 8, v[u]);
        }
      }
    }
  }
}

template <typename TX, typename TO>
static void lr_pad_launch(const LrFusedArgs &a, int fr, hipStream_t s) {
  const dim3 grid((unsigned)((a.T + fr - 1) / fr), (unsigned)a.B);
  auto go = [&](auto FRC) {
    constexpr int F = decltype(FRC)::value;
    if (a.pe != nullptr)
      hipLaunchKernelGGL((lr_pad_kernel<TX, TO, true, F>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((lr_pad_kernel<TX, TO, false, F>), grid, dim3(256), 0, s, a);
  };
  if (fr == 256)
    go(std::integral_constant<int, 256>{});
  else if (fr == 128)
    go(std::integral_constant<int, 128>{});
  else
    go(std::integral_constant<int, 64>{});
}

// The reference's LengthRegulator.forward + pad (modules.py:161-194, tools.py:360-378) in ONE launch:
// duration scan, gather (+ PE) into the padded [B, T_out, D] output, zeros past min(mel_len, T_out).
// (Round 1-5: fs2_lr_durations + fs2_lr_expand, two dependent launches.)
extern "C" int fs2_length_regulate(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control, int B,
                                   int L, int D, int T_out, const float *pe, void *out, int out_dtype, int32_t *cum,
                                   int64_t *mel_len, float *d_rounded, int32_t *index_map, fs2_stream_t stream) {
  if (x == nullptr || dur == nullptr || cum == nullptr || mel_len == nullptr) return FS2_EINVAL;
  if (dur_kind < FS2_DUR_I64 || dur_kind > FS2_DUR_LOGPRED) return FS2_EINVAL;
  if (dur_kind == FS2_DUR_LOGPRED && d_rounded == nullptr) return FS2_EINVAL;
  if (out == nullptr && index_map == nullptr) return FS2_EINVAL;
  if (B < 0 || L <= 0 || D <= 0 || (D & 7) != 0 || T_out < 0 || (int64_t)B * T_out > 0x7fffff00LL) return FS2_EINVAL;
  if (B == 0) return FS2_OK;
  if (T_out == 0 || L > kLdsCum || out == nullptr) {  // long phoneme rows / map only: the two-launch form
    const int rc = fs2_lr_durations(dur, dur_kind, d_control, B, L, cum, mel_len, d_rounded, stream);
    if (rc != FS2_OK || T_out == 0) return rc;
    return fs2_lr_expand(x, x_dtype, cum, mel_len, B, L, D, T_out, pe, out, out_dtype, index_map, nullptr, stream);
  }
  LrFusedArgs a{};
  a.x = x;
  a.dur = dur;
  a.dur_kind = dur_kind;
  a.d_control = d_control;
  a.B = B;
  a.L = L;
  a.D = D;
  a.T = T_out;
  a.pe = pe;
  a.out = out;
  a.cum = cum;
  a.mel_len = mel_len;
  a.d_rounded = d_rounded;
  a.padded = 1;
  a.index_map = index_map;
  if (L > 1024) return lr_fused_launch(a, x_dtype, out_dtype, as_stream(stream));
  // frames per workgroup: 128 once that still gives >= 2 workgroups per CU (cfg4: 2,048 of 64 KB),
  // else 64 (cfg2: 448 of 32 KB); FS2_LR_PAD_FR = 64 / 128 / 256 for A/B
  static const int fr_env = [] {
    const char *e = getenv("FS2_LR_PAD_FR");
    const int v = e != nullptr ? atoi(e) : 0;
    return (v == 64 || v == 128 || v == 256) ? v : 0;
  }();
  const int fr = fr_env != 0 ? fr_env : (int64_t)B * ((T_out + 127) / 128) >= 512 ? 128 : 64;
  hipStream_t s = as_stream(stream);
  if (x_dtype == FS2_BF16 && out_dtype == FS2_BF16)
    lr_pad_launch<bf16, bf16>(a, fr, s);
  else if (x_dtype == FS2_F32 && out_dtype == FS2_F32)
    lr_pad_launch<float, float>(a, fr, s);
  else if (x_dtype == FS2_F32 && out_dtype == FS2_BF16)
    lr_pad_launch<float, bf16>(a, fr, s);
  else if (x_dtype == FS2_BF16 && out_dtype == FS2_F32)
    lr_pad_launch<bf16, float>(a, fr, s);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_lr_backward(const float *dy, const int32_t *cum, int B, int L, int D, int T, float *dx,
                               fs2_stream_t stream) {
  if (dy == nullptr || cum == nullptr || dx == nullptr || B < 0 || L < 0 || T < 0 || D <= 0 || (D & 7) || D > 2048)
    return FS2_EINVAL;
  if (B == 0 || L == 0) return FS2_OK;
  hipLaunchKernelGGL(lr_bwd_kernel, dim3((unsigned)((L + 7) / 8), (unsigned)B), dim3(256), 0, as_stream(stream), dy,
                     cum, L, D, T, dx);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_len_stats(const int64_t *lens, int B, const int32_t *bad_counter, int32_t *meta, fs2_stream_t stream) {
  if (lens == nullptr || meta == nullptr || B < 0) return FS2_EINVAL;
  hipLaunchKernelGGL(len_stats_kernel, dim3(1), dim3(256), 0, as_stream(stream), lens, B, bad_counter, meta);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_lr_fused(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control,
                            const int32_t *cum_in, const int64_t *mel_len_in, int B, int L, int D, int T_out,
                            const float *pe, const int64_t *layout_lens, int32_t *cu, int32_t *row_pos,
                            int32_t *rowmap, void *out, int out_dtype, int32_t *cum, int64_t *mel_len,
                            float *d_rounded, fs2_stream_t stream) {
  return fs2_lr_fused_proj(x, x_dtype, dur, dur_kind, d_control, cum_in, mel_len_in, B, L, D, T_out, pe, layout_lens,
                           cu, row_pos, rowmap, out, out_dtype, cum, mel_len, d_rounded, nullptr, nullptr, 0, nullptr,
                           stream);
}

extern "C" int fs2_lr_fused_proj(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control,
                                 const int32_t *cum_in, const int64_t *mel_len_in, int B, int L, int D, int T_out,
                                 const float *pe, const int64_t *layout_lens, int32_t *cu, int32_t *row_pos,
                                 int32_t *rowmap, void *out, int out_dtype, int32_t *cum, int64_t *mel_len,
                                 float *d_rounded, const float *proj_src, const float *proj_pe, int NP,
                                 void *proj_out, fs2_stream_t stream) {
  if (proj_out != nullptr && (proj_src == nullptr || proj_pe == nullptr || NP < 8 || NP > 1536 || (NP & 7) != 0))
    return FS2_EINVAL;
  if (x == nullptr || out == nullptr || layout_lens == nullptr || cu == nullptr) return FS2_EINVAL;
  if (B < 0 || L <= 0 || D <= 0 || (D & 7) != 0 || T_out < 0 || B > kSeqMaxB || L > kLdsCum) return FS2_EINVAL;
  if ((int64_t)B * T_out > 0x7fffff00LL) return FS2_EINVAL;
  if (dur != nullptr) {  // scan mode: durations in, cum / mel_len out
    if (cum == nullptr || mel_len == nullptr || dur_kind < FS2_DUR_I64 || dur_kind > FS2_DUR_LOGPRED) return FS2_EINVAL;
    if (dur_kind == FS2_DUR_LOGPRED && d_rounded == nullptr) return FS2_EINVAL;
  } else if (cum_in == nullptr || mel_len_in == nullptr) {
    return FS2_EINVAL;
  }
  if (B == 0) return FS2_OK;
  if (T_out == 0) {
    // nothing to gather, but the scan outputs and cu are still due: one frame block of work
    if (dur != nullptr) {
      int rc = fs2_lr_durations(dur, dur_kind, d_control, B, L, cum, mel_len, d_rounded, stream);
      if (rc != FS2_OK) return rc;
    }
    return fs2_seq_layout(layout_lens, B, 0, cu, row_pos, rowmap, stream);
  }
  LrFusedArgs a{};
  a.x = x;
  a.dur = dur;
  a.dur_kind = dur_kind;
  a.d_control = d_control;
  a.cum_in = cum_in;
  a.mel_len_in = mel_len_in;
  a.lens = layout_lens;
  a.B = B;
  a.L = L;
  a.D = D;
  a.T = T_out;
  a.pe = pe;
  a.out = out;
  a.cum = cum;
  a.mel_len = mel_len;
  a.d_rounded = d_rounded;
  a.cu = cu;
  a.row_pos = reinterpret_cast<int2 *>(row_pos);
  a.rowmap = rowmap;
  static const int store_env = [] {
    const char *e = getenv("FS2_LR_STORE");
    return e == nullptr ? 0 : (e[0] == 'p' ? 1 : e[0] == 's' ? 2 : 0);
  }();
  a.store = store_env;
  a.proj_src = proj_src;
  a.proj_pe = proj_pe;
  a.NP = NP;
  a.proj_out = reinterpret_cast<bf16 *>(proj_out);
  return lr_fused_launch(a, x_dtype, out_dtype, as_stream(stream));
}

static int lr_fused_launch(const LrFusedArgs &a, int x_dtype, int out_dtype, hipStream_t s) {
  const int T_out = a.T, B = a.B;
  // frames per workgroup (FS2_LR_ROWS = 32 / 64 / 128, A/B): every workgroup re-derives its
  // utterance's scan and packed offset, so more frames per workgroup amortise that prologue
  static const int rows_env = [] {
    const char *e = getenv("FS2_LR_ROWS");
    const int v = e != nullptr ? atoi(e) : 32;
    return (v == 64 || v == 128) ? v : 32;
  }();
  const int R = rows_env;
  const dim3 grid((unsigned)((T_out + R - 1) / R), (unsigned)B);
  auto go = [&](auto TXv, auto TOv) {
    using TX = decltype(TXv);
    using TO = decltype(TOv);
    auto launch = [&](auto RC) {
      constexpr int RR = decltype(RC)::value;
      if (a.pe != nullptr)
        hipLaunchKernelGGL((lr_fused_kernel<TX, TO, true, RR>), grid, dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((lr_fused_kernel<TX, TO, false, RR>), grid, dim3(256), 0, s, a);
    };
    if (R == 128)
      launch(std::integral_constant<int, 128>{});
    else if (R == 64)
      launch(std::integral_constant<int, 64>{});
    else
      launch(std::integral_constant<int, 32>{});
  };
  if (x_dtype == FS2_BF16 && out_dtype == FS2_BF16)
    go(bf16{}, bf16{});
  else if (x_dtype == FS2_F32 && out_dtype == FS2_F32)
    go(0.0f, 0.0f);
  else if (x_dtype == FS2_F32 && out_dtype == FS2_BF16)
    go(0.0f, bf16{});
  else if (x_dtype == FS2_BF16 && out_dtype == FS2_F32)
    go(bf16{}, 0.0f);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
