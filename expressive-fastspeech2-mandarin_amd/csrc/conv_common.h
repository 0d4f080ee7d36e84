// Shared pieces of the implicit-GEMM conv kernels (conv_gemm.hip) and the fused FFN kernel
// (ffn.hip): buffer-resource loads, the swizzled 128-byte LDS row, the kernel argument block and
// the LDS epilogues (bias / activation / residual / LayerNorm + mask) of a BM x BN f32 tile.
#pragma once
#include <cstdlib>

#include "fs2_common.h"

namespace {

constexpr int kRowBytes = 128;  // one k-step of one tile row

__device__ __forceinline__ int lds_off(int row, int chunk) { return row * kRowBytes + ((chunk ^ (row & 7)) << 4); }

// fp8 fragment of mfma_scale_f32_16x16x128_f8f6f4: lane group g = lane>>4 holds k = 32g .. 32g+31
// of its row (16-byte chunks 2g and 2g+1 of the 128-byte k-step row); A and B use the same map.
__device__ __forceinline__ i32x8 frag_fp8(const char *p0, const char *p1) {
  const uint4 lo = *reinterpret_cast<const uint4 *>(p0), hi = *reinterpret_cast<const uint4 *>(p1);
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}
__device__ __forceinline__ f32x4 mfma_fp8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);  // e4m3 x e4m3, scale 1
}

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
template <>
struct CTraits<FS2_FP8> {
  static constexpr int KE = 128;  // one mfma_scale_f32_16x16x128_f8f6f4 per k-step
  static constexpr int CE = 16;
  using T = fp8;
};

// One 16-byte LDS chunk (CE compute elements) staged in registers from an input of type TIn.
// Loads are raw buffer loads: an out-of-range byte offset (kOOB) returns zeros in hardware, so
// the conv's zero padding / tile edges cost a select on the offset instead of a branch per load
// (branches around loads make hipcc wait vmcnt(0) per element, serialising the stage).
constexpr uint32_t kOOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
// a 16-byte output store, write-through (sc1: the line leaves the XCD's L2 instead of staying dirty
// there; measured 1-3 % faster kernels downstream) or plain; `base` must be wave-uniform
__device__ __forceinline__ void store16_out(void *base, uint32_t off, uint4 v, int sc1) {
  if (sc1)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                           make_rsrc(base, 0x7fffffffu), off, 0, 16);
  else
    *reinterpret_cast<uint4 *>(static_cast<char *>(base) + off) = v;
}
// FS2_OUT_SC1=0 turns the write-through output stores off (A/B); read once per library
static inline int env_out_sc1() {
  static const int v = [] {
    const char *e = getenv("FS2_OUT_SC1");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  return v;
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint2 bload8(rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v[0], v[1]);
}

template <int CT, typename TIn>
struct Stage;
template <>
struct Stage<FS2_BF16, bf16> {
  uint4 r;
  __device__ __forceinline__ void load(rsrc_t rs, uint32_t off) { r = bload16(rs, off); }
  __device__ __forceinline__ uint4 chunk() const { return r; }
};
template <>
struct Stage<FS2_BF16, float> {
  uint4 a, b;
  __device__ __forceinline__ void load(rsrc_t rs, uint32_t off) {
    a = bload16(rs, off);
    b = bload16(rs, off + 16u);
  }
  __device__ __forceinline__ uint4 chunk() const {
    bf16x8 v = {(bf16)__uint_as_float(a.x), (bf16)__uint_as_float(a.y), (bf16)__uint_as_float(a.z),
                (bf16)__uint_as_float(a.w), (bf16)__uint_as_float(b.x), (bf16)__uint_as_float(b.y),
                (bf16)__uint_as_float(b.z), (bf16)__uint_as_float(b.w)};
    return *reinterpret_cast<uint4 *>(&v);
  }
};
template <>
struct Stage<FS2_F32, float> {
  uint4 r;
  __device__ __forceinline__ void load(rsrc_t rs, uint32_t off) { r = bload16(rs, off); }
  __device__ __forceinline__ uint4 chunk() const { return r; }
};
template <>
struct Stage<FS2_F32, bf16> {
  uint2 r;
  __device__ __forceinline__ void load(rsrc_t rs, uint32_t off) { r = bload8(rs, off); }
  __device__ __forceinline__ uint4 chunk() const {
    return make_uint4(r.x << 16, r.x & 0xffff0000u, r.y << 16, r.y & 0xffff0000u);
  }
};

template <>
struct Stage<FS2_FP8, fp8> {
  uint4 r;
  __device__ __forceinline__ void load(rsrc_t rs, uint32_t off) { r = bload16(rs, off); }
  __device__ __forceinline__ uint4 chunk() const { return r; }
};

struct ConvArgs {
  const void *x;
  int64_t xs;
  const void *w;
  const float *bias;
  int B, T, Cin, Cin_pad, N, KS, pad, M;
  int ntn;  // number of N tiles
  int ngr;  // N tiles per group in the tile order (== ntn: N-fastest over the whole row)
  uint32_t x_bytes, w_bytes;
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
  // packed rows (NULL = padded [B, T] rows): active row count = *rows_dev, row r is frame
  // row_pos[2r] of a sequence of length row_pos[2r+1]
  const int32_t *rows_dev;
  const int2 *row_pos;
  const int32_t *a_rowmap;  // KS == 1 only: A row of output row m (-1 = zero row)
  int dbg;  // analysis only (FS2_CONV_DEBUG): bit 0 skips the K loop, bit 1 the epilogue; LN epilogue
            // ablations: bit 2 no stores, bit 3 no residual loads, bit 4 no row reductions
  const float *colscale;    // fp8: per-column dequantisation scale of the accumulator (or NULL)
  float out_scale;          // out_dt == FS2_FP8: e4m3(y * out_scale)
  void *out2;               // optional copy, rows of N: LN epilogues e4m3(y * out2_scale), others bf16(y)
  float out2_scale;
  int cin_block;            // split-precision input: logical channel blocks of cin_block (0 = off)
  int cin_src[4];           // ... block i is source channel cin_src[i] of x
  int out_split;            // LN epilogue: bf16 hi plane at column n, lo plane at column N + n
  // split-K tail (conv_gemm_kernel, LDS-DMA path): see conv_tile_sk. sk_slots = 0 disables it.
  int sk_slots;             // workgroups resident at once (CUs x workgroups per CU)
  int sk_max;               // most segments one tail tile may be split into
  int *sk_cnt;              // [sk_slots] arrival counters (zero between launches; self-resetting)
  float *sk_part;           // [sk_slots][BM*BN] f32 partial tiles
  uint32_t sk_part_bytes;
  int64_t sk_ws_bytes;      // host side only: workspace size
  // Row split between the phased 256x256 kernel and the 128x128 kernel (split_rows): 0 = off,
  // 1 = this launch runs the 256-row panels [0, P1), 2 = it runs the rows from P1 * 256 on.
  int row_split;
  int split_slots;          // workgroups the phased kernel runs at once (one per CU)
  int ln_pairs;             // LayerNorm epilogues: two rows per wave-iteration, 16-byte stores
  // vocoder extensions (fs2_conv_desc): dilated taps, leaky-ReLU epilogue / out2 activation,
  // two-addend residual sum with a final divisor
  int dil;
  float slope, slope2;
  int out2_act, out2_f32;
  const void *res2;
  float out_div;
  int l2pf;  // ring kernel: warm each XCD's L2 with the whole weight matrix before the K loop
  int group_n, group_cin;  // grouped input: columns [g*group_n, ...) read channels + g*group_cin
};

constexpr int64_t kSkCntBytes = 4096;  // counter block at the start of the split-K workspace

// Source channel of logical input channel c (split-precision layouts map channel blocks).
__device__ __forceinline__ int src_channel(const ConvArgs &a, int c) {
  if (a.cin_block == 0) return c;
  const int blk = c / a.cin_block;
  return a.cin_src[blk] + (c - blk * a.cin_block);
}

__device__ __forceinline__ void load_any4(const void *p, int dt, int64_t off, float v[4]) {
  if (dt == FS2_BF16)
    load4(reinterpret_cast<const bf16 *>(p) + off, v);
  else
    load4(reinterpret_cast<const float *>(p) + off, v);
}
__device__ __forceinline__ void store_any4(void *p, int dt, int64_t off, const float v[4], float scale = 1.0f) {
  if (dt == FS2_BF16)
    store4(reinterpret_cast<bf16 *>(p) + off, v);
  else if (dt == FS2_FP8)
    *reinterpret_cast<unsigned *>(reinterpret_cast<fp8 *>(p) + off) = pack4_fp8(v, scale);
  else
    store4(reinterpret_cast<float *>(p) + off, v);
}

// Epilogue of one BM x BN tile whose f32 accumulators sit in LDS (E, row stride BN + 4).
// (Prefetching every row's residual before the LN row loop was measured 3-5 % slower on the
// LN GEMMs in round 1: more registers, and the row loop is not latency-bound.)
// Residual rows of the paired LayerNorm epilogue (RES_LN): lane (wave wid, half h, column group
// hl) loads row m0 + wid + (2p + h) * NWAVES, 8 columns (one uint4 of bf16 or two of f32).
// (Issuing them before the ring kernel's K loop instead -- untracked asm loads, waited after it --
// measured fc + LN 16.4 -> 16.0 us: not kept.)
template <int NP, int NWAVES>
__device__ __forceinline__ void load_res_pairs(const ConvArgs &a, int m0, int M, int tid, uint4 (&rraw)[NP][2]) {
  const int lane = tid & 63, wid = tid >> 6, h = lane >> 5, n = (lane & 31) * 8;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int m = min(m0 + wid + (2 * p + h) * NWAVES, M - 1);
    if (a.res_dt == FS2_BF16) {
      rraw[p][0] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const bf16 *>(a.res) + (int64_t)m * a.rs + n);
      rraw[p][1] = rraw[p][0];
    } else {
      const uint4 *rp = reinterpret_cast<const uint4 *>(reinterpret_cast<const float *>(a.res) + (int64_t)m * a.rs + n);
      rraw[p][0] = rp[0];
      rraw[p][1] = rp[1];
    }
  }
}

template <int BM, int BN, int NWAVES, bool LN = true>
__device__ __forceinline__ void epilogue(const ConvArgs &a, const float *E, int m0, int n0, int tid, int M) {
  constexpr int EPI_LD = BN + 4;
  const int lane = tid & 63, wid = tid >> 6;
  const int T = a.T;
  const int epi = a.epi;
  static_assert(BM % NWAVES == 0, "rows per wave");
  if constexpr (LN && (BM / NWAVES) % 2 == 0) if (a.ln_pairs && (epi == FS2_EPI_RES_LN || epi == FS2_EPI_RELU_LN ||
                                                                  epi == FS2_EPI_RELU_LN_DOT)) {
    // Two rows per wave-iteration: half-wave h = lane >> 5 takes row k = 2p + h of the wave's rows,
    // lane owns columns 8*(lane & 31) .. +7 (N == BN == 256). 16-byte residual loads and output
    // stores (8-byte ones are issue-bound), half the reduction chains of one row per wave.
    constexpr int RPW = BM / NWAVES, NP = RPW / 2;
    const int h = lane >> 5, hl = lane & 31;
    const int n = hl * 8;
    float bias8[8], g8[8], be8[8], cs8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    load8(a.gamma + n, g8);
    load8(a.beta + n, be8);
    load8(a.bias + n, bias8);
    if (a.colscale != nullptr) load8(a.colscale + n, cs8);
    const float inv_n = 1.0f / (float)a.N;
    auto hsum = [](float v) {  // sum over the 32 lanes of a half-wave
      v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
      v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
      v += dpp_mov<0x141>(v);  // row_half_mirror
      v += dpp_mov<0x140>(v);  // row_mirror: every lane of a 16-lane row holds the row's sum
      return v + __shfl_xor(v, 16, 64);
    };
    const bool res_bf16 = a.res_dt == FS2_BF16;
    uint4 rraw[NP][2];
    if (epi == FS2_EPI_RES_LN && (a.dbg & 8)) {  // analysis: no residual loads
#pragma unroll
      for (int p = 0; p < NP; ++p) rraw[p][0] = rraw[p][1] = make_uint4(0u, 0u, 0u, 0u);
    } else if (epi == FS2_EPI_RES_LN) {
      load_res_pairs<NP, NWAVES>(a, m0, M, tid, rraw);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        asm volatile("" ::"v"(rraw[p][0].x), "v"(rraw[p][0].y), "v"(rraw[p][0].z), "v"(rraw[p][0].w),
                     "v"(rraw[p][1].x), "v"(rraw[p][1].y), "v"(rraw[p][1].z), "v"(rraw[p][1].w));
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = wid + (2 * p + h) * NWAVES;
      const bool row_ok = m0 + r < M;
      const int m = min(m0 + r, M - 1);
      float v[8];
      load8(E + r * EPI_LD + n, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * cs8[q] + bias8[q];
      if (epi == FS2_EPI_RES_LN) {
        if (res_bf16) {
          const uint32_t w4[4] = {rraw[p][0].x, rraw[p][0].y, rraw[p][0].z, rraw[p][0].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] += __uint_as_float(w4[q] << 16);
            v[2 * q + 1] += __uint_as_float(w4[q] & 0xffff0000u);
          }
        } else {
          const uint32_t w8[8] = {rraw[p][0].x, rraw[p][0].y, rraw[p][0].z, rraw[p][0].w,
                                  rraw[p][1].x, rraw[p][1].y, rraw[p][1].z, rraw[p][1].w};
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] += __uint_as_float(w8[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.0f);
      }
      float s1 = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) s1 += v[q];
      const bool nored = (a.dbg & 16) != 0;  // analysis: lane-local statistics (no shuffles)
      const float mean = (nored ? s1 : hsum(s1)) * inv_n;
      float d[8], ss = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        d[q] = v[q] - mean;
        ss += d[q] * d[q];
      }
      const float var = (nored ? ss : hsum(ss)) * inv_n;
      const float rstd = 1.0f / sqrtf(var + a.eps);
      float y[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = d[q] * rstd * g8[q] + be8[q];
      const int bb = m / T;
      const int t = m - bb * T;
      const bool masked = (a.lens != nullptr) && ((int64_t)t >= a.lens[bb]);
      if (epi == FS2_EPI_RELU_LN_DOT) {
        float dw8[8];
        load8(a.dw + n, dw8);
        float sd = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) sd += y[q] * dw8[q];
        const float sdot = hsum(sd) + a.db;
        if (hl == 0 && row_ok) reinterpret_cast<float *>(a.out)[m] = masked ? 0.0f : sdot;
        continue;
      }
      if (epi == FS2_EPI_RES_LN) {
        if (masked) {
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] = 0.0f;
        }
        if (a.av1 != nullptr) {
          float av[8];
          load8(a.av1 + (int64_t)bb * a.N + n, av);
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] += av[q];
        }
        if (a.av2 != nullptr) {
          float av[8];
          load8(a.av2 + (int64_t)bb * a.N + n, av);
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] += av[q];
        }
      }
      if (!row_ok) continue;
      if (a.dbg & 4) {  // analysis: no output stores
        asm volatile("" ::"v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]), "v"(y[6]), "v"(y[7]));
        continue;
      }
      if (a.out_split) {  // two bf16 planes: hi, lo = bf16(y - hi)
        float hi[8], lo[8];
        bf16 *op = reinterpret_cast<bf16 *>(a.out) + (int64_t)m * a.os;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          hi[q] = (float)(bf16)y[q];
          lo[q] = y[q] - hi[q];
        }
        store8(op + n, hi);
        store8(op + a.N + n, lo);
        continue;
      }
      if (a.out_dt == FS2_BF16)
        store8(reinterpret_cast<bf16 *>(a.out) + (int64_t)m * a.os + n, y);
      else if (a.out_dt == FS2_F32)
        store8(reinterpret_cast<float *>(a.out) + (int64_t)m * a.os + n, y);
      else {
        uint2 o = make_uint2(pack4_fp8(y, a.out_scale), pack4_fp8(y + 4, a.out_scale));
        *reinterpret_cast<uint2 *>(reinterpret_cast<fp8 *>(a.out) + (int64_t)m * a.os + n) = o;
      }
      if (a.out2 != nullptr) {
        uint2 o = make_uint2(pack4_fp8(y, a.out2_scale), pack4_fp8(y + 4, a.out2_scale));
        *reinterpret_cast<uint2 *>(reinterpret_cast<fp8 *>(a.out2) + (int64_t)m * a.N + n) = o;
      }
    }
    return;
  }
  if constexpr (LN) if (epi == FS2_EPI_RES_LN || epi == FS2_EPI_RELU_LN || epi == FS2_EPI_RELU_LN_DOT) {
    // one wave per row; N == BN == 256 (checked on the host), lane owns columns 4*lane..4*lane+3
    const int n = lane * 4;
    float bias4[4], g4[4], be4[4], cs4[4] = {1.f, 1.f, 1.f, 1.f};
    load4(a.gamma + n, g4);
    load4(a.beta + n, be4);
#pragma unroll
    for (int q = 0; q < 4; ++q) bias4[q] = a.bias[n + q];
    if (a.colscale != nullptr) load4(a.colscale + n, cs4);
    const float inv_n = 1.0f / (float)a.N;
    // Residual rows of ALL this wave's rows are loaded before the first row is reduced, and the
    // empty asm consuming them pins the loads there (otherwise they are scheduled next to their
    // use: one dependent memory latency per row, 16 per tile on the decoder shapes).
    static_assert(BM % NWAVES == 0, "rows per wave");
    constexpr int RPW = BM / NWAVES;
    uint4 rraw[RPW];
    const bool res_bf16 = a.res_dt == FS2_BF16;
    if (epi == FS2_EPI_RES_LN && (a.dbg & 8)) {
#pragma unroll
      for (int i = 0; i < RPW; ++i) rraw[i] = make_uint4(0u, 0u, 0u, 0u);
    } else if (epi == FS2_EPI_RES_LN) {
      if (res_bf16) {
        const bf16 *rp = reinterpret_cast<const bf16 *>(a.res);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int m = min(m0 + wid + i * NWAVES, M - 1);
          const uint2 u = *reinterpret_cast<const uint2 *>(rp + (int64_t)m * a.rs + n);
          rraw[i] = make_uint4(u.x, u.y, 0u, 0u);
        }
      } else {
        const float *rp = reinterpret_cast<const float *>(a.res);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int m = min(m0 + wid + i * NWAVES, M - 1);
          rraw[i] = *reinterpret_cast<const uint4 *>(rp + (int64_t)m * a.rs + n);
        }
      }
#pragma unroll
      for (int i = 0; i < RPW; ++i) asm volatile("" ::"v"(rraw[i].x), "v"(rraw[i].y), "v"(rraw[i].z), "v"(rraw[i].w));
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wid + i * NWAVES;
      // rows past M are computed on clamped data and not stored: no control dependency between
      // rows, so the compiler can interleave their (latency-bound) reduction chains
      const bool row_ok = m0 + r < M;
      const int m = min(m0 + r, M - 1);
      float v[4];
      load4(E + r * EPI_LD + n, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = v[q] * cs4[q] + bias4[q];
      if (epi == FS2_EPI_RES_LN) {
        float rv[4];
        if (res_bf16) {
          rv[0] = __uint_as_float(rraw[i].x << 16);
          rv[1] = __uint_as_float(rraw[i].x & 0xffff0000u);
          rv[2] = __uint_as_float(rraw[i].y << 16);
          rv[3] = __uint_as_float(rraw[i].y & 0xffff0000u);
        } else {
          rv[0] = __uint_as_float(rraw[i].x);
          rv[1] = __uint_as_float(rraw[i].y);
          rv[2] = __uint_as_float(rraw[i].z);
          rv[3] = __uint_as_float(rraw[i].w);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += rv[q];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.0f);
      }
      const bool nored = (a.dbg & 16) != 0;
      const float mean = (nored ? (v[0] + v[1] + v[2] + v[3]) : wave_sum(v[0] + v[1] + v[2] + v[3])) * inv_n;
      float d[4], ss = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[q] = v[q] - mean;
        ss += d[q] * d[q];
      }
      const float var = (nored ? ss : wave_sum(ss)) * inv_n;
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
        if (lane == 0 && row_ok) reinterpret_cast<float *>(a.out)[m] = masked ? 0.0f : s;
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
      if (a.dbg & 4) {
        asm volatile("" ::"v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]));
        continue;
      }
      if (!row_ok) continue;
      if (a.out_split) {  // two bf16 planes: hi, lo = bf16(y - hi)
        float hi[4], lo[4];
        bf16 *op = reinterpret_cast<bf16 *>(a.out) + (int64_t)m * a.os;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          hi[q] = (float)(bf16)y[q];
          lo[q] = y[q] - hi[q];
        }
        store4(op + n, hi);
        store4(op + a.N + n, lo);
        continue;
      }
      store_any4(a.out, a.out_dt, (int64_t)m * a.os + n, y, a.out_scale);
      if (a.out2 != nullptr)
        *reinterpret_cast<unsigned *>(reinterpret_cast<fp8 *>(a.out2) + (int64_t)m * a.N + n) = pack4_fp8(y, a.out2_scale);
    }
    return;
  }

  constexpr int NT = 64 * NWAVES;
  if ((a.N & 7) == 0 && (a.os & 7) == 0 && a.ln_pairs && a.out_dt != FS2_F32) {
    // elementwise epilogues with bf16 / fp8 outputs, 8 columns per thread: 16-byte stores (8-byte
    // ones are issue-bound on the store-heavy launches: Q|K|V writes 3x what it reads). f32
    // outputs keep the 4-column path below, whose stores are 16 bytes already.
    constexpr int G8 = BN / 8;
    static_assert(NT % G8 == 0, "column group per thread");
    const int cg = tid % G8;
    const int n = n0 + cg * 8;
    if (n >= a.N) return;
    float bias8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, cs8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    if (a.bias != nullptr) load8(a.bias + n, bias8);
    if (a.colscale != nullptr) load8(a.colscale + n, cs8);
    for (int r = tid / G8; r < BM; r += NT / G8) {
      const int m = m0 + r;
      if (m >= M) break;
      float v[8];
      load8(E + r * EPI_LD + cg * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * cs8[q] + bias8[q];
      if (epi == FS2_EPI_BIAS_RELU) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.0f);
      } else if (epi == FS2_EPI_BIAS_TANH) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = tanhf(v[q]);
      } else if (epi == FS2_EPI_BIAS_RES || epi == FS2_EPI_RES_SUM) {
        float rv[8];
        load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
        load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n + 4, rv + 4);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += rv[q];
        if (epi == FS2_EPI_RES_SUM) {
          if (a.res2 != nullptr) {
            load_any4(a.res2, a.out_dt, (int64_t)m * a.os + n, rv);
            load_any4(a.res2, a.out_dt, (int64_t)m * a.os + n + 4, rv + 4);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += rv[q];
          }
          if (a.out_div != 1.0f) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = v[q] / a.out_div;
          }
        }
      } else if (epi == FS2_EPI_BIAS_LRELU) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.0f ? v[q] : v[q] * a.slope;
      } else if (epi == FS2_EPI_RELU_GRAD) {
        float rv[8];
        load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
        load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n + 4, rv + 4);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = rv[q] > 0.0f ? v[q] : 0.0f;
      }
      const int64_t o = (int64_t)m * a.os + n;
      if (a.out_dt == FS2_BF16)
        store8(reinterpret_cast<bf16 *>(a.out) + o, v);
      else if (a.out_dt == FS2_F32)
        store8(reinterpret_cast<float *>(a.out) + o, v);
      else
        *reinterpret_cast<uint2 *>(reinterpret_cast<fp8 *>(a.out) + o) =
            make_uint2(pack4_fp8(v, a.out_scale), pack4_fp8(v + 4, a.out_scale));
      if (a.out2 != nullptr) {
        if (a.out2_act) {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.0f ? v[q] : v[q] * a.slope2;
        }
        if (a.out2_f32)
          store8(reinterpret_cast<float *>(a.out2) + (int64_t)m * a.N + n, v);
        else
          store8(reinterpret_cast<bf16 *>(a.out2) + (int64_t)m * a.N + n, v);
      }
    }
    return;
  }
  // elementwise epilogues: each thread keeps one 4-column group (threads % (BN/4) == 0), so its
  // bias is loaded once; rows step by threads / (BN/4)
  constexpr int G = BN / 4;
  static_assert(NT % G == 0, "column group per thread");
  const int cg = tid % G;
  const int n = n0 + cg * 4;
  if (n >= a.N) return;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f}, cs4[4] = {1.f, 1.f, 1.f, 1.f};
  if (a.bias != nullptr) load4(a.bias + n, bias4);
  if (a.colscale != nullptr) load4(a.colscale + n, cs4);
  for (int r = tid / G; r < BM; r += NT / G) {
    const int m = m0 + r;
    if (m >= M) break;
    float v[4];
    load4(E + r * EPI_LD + cg * 4, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = v[q] * cs4[q] + bias4[q];
    if (epi == FS2_EPI_BIAS_RELU) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.0f);
    } else if (epi == FS2_EPI_BIAS_TANH) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
    } else if (epi == FS2_EPI_BIAS_RES || epi == FS2_EPI_RES_SUM) {
      float rv[4];
      load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += rv[q];
      if (epi == FS2_EPI_RES_SUM) {
        if (a.res2 != nullptr) {
          load_any4(a.res2, a.out_dt, (int64_t)m * a.os + n, rv);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += rv[q];
        }
        if (a.out_div != 1.0f) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = v[q] / a.out_div;
        }
      }
    } else if (epi == FS2_EPI_BIAS_LRELU) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.0f ? v[q] : v[q] * a.slope;
    } else if (epi == FS2_EPI_RELU_GRAD) {
      float rv[4];
      load_any4(a.res, a.res_dt, (int64_t)m * a.rs + n, rv);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = rv[q] > 0.0f ? v[q] : 0.0f;
    }
    store_any4(a.out, a.out_dt, (int64_t)m * a.os + n, v, a.out_scale);
    if (a.out2 != nullptr) {
      if (a.out2_act) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.0f ? v[q] : v[q] * a.slope2;
      }
      if (a.out2_f32)
        store4(reinterpret_cast<float *>(a.out2) + (int64_t)m * a.N + n, v);
      else
        store4(reinterpret_cast<bf16 *>(a.out2) + (int64_t)m * a.N + n, v);
    }
  }
}

// Wait until at most n of this wave's vector-memory loads are outstanding (n wave-uniform, < 16).
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

}  // namespace
