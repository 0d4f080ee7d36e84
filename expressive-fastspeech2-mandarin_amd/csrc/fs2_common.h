// Shared device helpers for the fs2 HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fs2hip.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define FS2_WAVE 64

#define FS2_CHECK_LAUNCH()                                                                       \
  do {                                                                                           \
    hipError_t _e = hipGetLastError();                                                           \
    if (_e != hipSuccess) return FS2_ELAUNCH;                                                    \
  } while (0)

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }

// 8 consecutive elements -> 8 floats
__device__ __forceinline__ void load8(const float *p, float v[8]) {
  float4 a = reinterpret_cast<const float4 *>(p)[0];
  float4 b = reinterpret_cast<const float4 *>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16 *p, float v[8]) {
  uint4 r = *reinterpret_cast<const uint4 *>(p);
  uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(float *p, const float v[8]) {
  reinterpret_cast<float4 *>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4 *>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store8(bf16 *p, const float v[8]) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
  *reinterpret_cast<bf16x8 *>(p) = o;
}
__device__ __forceinline__ void store4(float *p, const float v[4]) {
  *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void store4(bf16 *p, const float v[4]) {
  bf16x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (bf16)v[i];
  *reinterpret_cast<bf16x4 *>(p) = o;
}
__device__ __forceinline__ void load4(const float *p, float v[4]) {
  float4 a = *reinterpret_cast<const float4 *>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
__device__ __forceinline__ void load4(const bf16 *p, float v[4]) {
  uint2 r = *reinterpret_cast<const uint2 *>(p);
  v[0] = __uint_as_float(r.x << 16);
  v[1] = __uint_as_float(r.x & 0xffff0000u);
  v[2] = __uint_as_float(r.y << 16);
  v[3] = __uint_as_float(r.y & 0xffff0000u);
}

// fp8 e4m3fn (OCP, the gfx950 MFMA format) as raw bytes. Conversion saturates to +-448 first
// (the hardware conversion does not clamp); 4 values -> one 32-bit word, element 0 in byte 0.
typedef unsigned char fp8;
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ unsigned pack4_fp8(const float v[4], float scale) {
  float c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = fminf(fmaxf(v[q] * scale, -448.0f), 448.0f);
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], r, true);
  return (unsigned)r;
}

// Full-wave sum, result in every lane. Within each 16-lane row: DPP quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror, row_mirror (VALU ops, no LDS round trip); the four row sums are
// then combined with v_readlane into a wave-uniform value. (A __shfl_xor butterfly is six
// dependent ds_bpermute LDS round trips: the LN epilogues' per-row critical path.)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline hipStream_t as_stream(fs2_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
