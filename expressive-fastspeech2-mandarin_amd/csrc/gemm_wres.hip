// Weight-resident projection GEMM for short-K, wide-N Linear / Conv1d(k=1) launches on many rows:
// the decoder's fused Q|K|V projection (M = 24.9k packed frames, K = 256, N = 768; SubLayers.py
// :39-41) and the encoder's (M = 4k).
//
// As 128 x 128 tiles those launches run ~1,200 short-K tiles in ~3 rounds, each paying its own
// load latency, 4 k-steps and epilogue (29 us for 51 MB of HBM traffic: 1.8 TB/s). Here every
// workgroup owns one 128-column slice of W for the whole launch and streams its share of the
// rows through a ring of 64-row A tiles (LDS-DMA,
// counted vmcnt, raw barrier: 2 tiles in flight while one computes) beside the W slice, which is
// DMA'd into LDS once (K = 256: 64 KiB). The MFMA takes W as the A operand, so each lane's accumulator holds 4 consecutive output COLUMNS of one row and the
// epilogue stores straight from registers (8-byte bf16x4 per lane, no LDS round trip).
// Grid: (N / 128) column slices x (CUs / slices) row workers, one workgroup per CU; the slices of
// one worker are adjacent after the XCD remap, so they share its A rows through one L2.
#include <cstdlib>

#include "gemm_wres.h"

namespace {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

__device__ __forceinline__ void vm_wait_n(int n) {  // n wave-uniform; >= 40 waits for 40
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
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 33: asm volatile("s_waitcnt vmcnt(33)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 35: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
    case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 37: asm volatile("s_waitcnt vmcnt(37)" ::: "memory"); break;
    case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 39: asm volatile("s_waitcnt vmcnt(39)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
  }
}

constexpr int kBM = 64, kBN = 128;  // A tile rows, slice columns
constexpr int kLDS = 160 * 1024;

// KSTEPS = K / 64 (one k-step = 64 bf16 = one 128-byte LDS row per tile row)
template <int KSTEPS>
__global__ __launch_bounds__(512, 1) void gemm_wres_kernel(WresArgs a, int nslice, int workers) {
  constexpr int WB = KSTEPS * kBN * 128;  // the W slice image (K = 256: 64 KiB)
  constexpr int AB = KSTEPS * kBM * 128;  // one A tile image
  constexpr int NA = (kLDS - WB) / AB;    // A ring depth: NA - 1 tiles in flight (K = 256: 3)
  constexpr int WMI = 2, NI = 2;          // wave: 32 rows x 32 columns
  constexpr int LA = KSTEPS;              // A pieces (1 KiB) per wave per tile
  constexpr int ST = WMI * NI;            // 8-byte stores per wave per tile
  __shared__ __attribute__((aligned(16))) char smem[WB + NA * AB];

  const int nwg = nslice * workers;
  const int bid = blockIdx.x;
  if (bid >= nwg) return;
  const int q = nwg >> 3, rem = nwg & 7, xcd = bid & 7, li = bid >> 3;
  const int g = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + li;  // bijective XCD remap
  const int slice = g % nslice, worker = g / nslice;
  const int n0 = slice * kBN;
  const int M = a.rows_dev != nullptr ? *a.rows_dev : a.M;
  const int TT = (M + kBM - 1) / kBM;
  const int t0 = (int)((int64_t)worker * TT / workers), t1 = (int)((int64_t)(worker + 1) * TT / workers);
  const int nt = t1 - t0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  // bias: loaded and waited for before the LDS-DMA ring starts (a tracked load in flight beside
  // it would make hipcc drain vmcnt to 0 at its first use)
  float bias4[NI][4];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int n = n0 + wc * 32 + ni * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) bias4[ni][j] = a.bias != nullptr ? a.bias[n + j] : 0.0f;
  }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
    asm volatile("" ::"v"(bias4[ni][0]), "v"(bias4[ni][1]), "v"(bias4[ni][2]), "v"(bias4[ni][3]));

  const rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.x), (short)0, (int)a.x_bytes, 0x00020000);
  // one 1 KiB piece = 8 rows x 128 B per wave instruction; lane l lands at row 8p + l/8, physical
  // chunk l&7, so it fetches logical chunk (l&7) ^ (row&7) (swizzle applied on the source)
  const int prow = lane >> 3, plc = (lane & 7) ^ prow;
  // the W slice: KSTEPS x 16 pieces of 8 columns x 128 B, 2 * KSTEPS per wave, once per launch
  const rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.w), (short)0, (int)a.w_bytes, 0x00020000);
  const uint32_t wrow = (uint32_t)a.K * 2u;
#pragma unroll
  for (int i = 0; i < 2 * KSTEPS; ++i) {
    const int p = wid + 8 * i, s = p >> 4, pq = p & 15;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        wrs, (__attribute__((address_space(3))) void *)(smem + s * (kBN * 128) + pq * 1024), 16,
        (uint32_t)(n0 + 8 * pq + prow) * wrow + (uint32_t)(s * 128 + plc * 16), 0, 0, 0);
  }
  const uint32_t xrow = (uint32_t)a.xs * 2u;
  auto dma_a = [&](int t, int buf) {  // tile t (absolute): rows 8*wid + l/8 of it, every k-step
    const int m = t * kBM + 8 * wid + prow;
    const bool ok = m < M;
    char *dst = smem + WB + buf * AB + wid * 1024;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(dst + s * (kBM * 128)),
                                               16, ok ? (uint32_t)m * xrow + (uint32_t)(s * 128 + plc * 16) : kOOB,
                                               0, 0, 0);
  };
  for (int j = 0; j < NA - 1 && j < nt; ++j) dma_a(t0 + j, j);

  const int aread = lds_off(wr * 32 + (lane & 15), lane >> 4);  // + mi * 16 rows; sub 1: + 4 chunks
  const int aread1 = lds_off(wr * 32 + (lane & 15), 4 + (lane >> 4));
  const int wread = lds_off(wc * 32 + (lane & 15), lane >> 4);  // + ni * 16 rows
  const int wread1 = lds_off(wc * 32 + (lane & 15), 4 + (lane >> 4));
  bf16 *out = reinterpret_cast<bf16 *>(a.out);

  int buf = 0;
  for (int i = 0; i < nt; ++i) {
    // tile i's A landed: the VMEM instructions this wave issued after dma_a(tile i) may stay in
    // flight (they retire in issue order) -- the prologue DMAs after it, then per tile j < i the
    // refill of tile j + NA - 1 (issued at j's top, j > i - NA + 1) and j's stores
    int cnt = 0;
    if (i < NA - 1) cnt += LA * (min(NA - 1, nt) - 1 - i);
    for (int j = max(0, i - NA + 1); j < i; ++j) cnt += ST + ((j > i - NA + 1 && j + NA - 1 < nt) ? LA : 0);
    vm_wait_n(cnt);
    __builtin_amdgcn_s_barrier();
    // refill the buffer tile i-1 used (every wave is past its reads: the barrier above)
    if (i + NA - 1 < nt) dma_a(t0 + i + NA - 1, buf == 0 ? NA - 1 : buf - 1);
    const char *As = smem + WB + buf * AB;
    f32x4 acc[NI][WMI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int mi = 0; mi < WMI; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const char *Xs = As + ks * (kBM * 128);
      const char *Ws = smem + ks * (kBN * 128);
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        bf16x8 xf[WMI], wf[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          wf[ni] = *reinterpret_cast<const bf16x8 *>(Ws + (sub ? wread1 : wread) + ni * 16 * 128);
#pragma unroll
        for (int mi = 0; mi < WMI; ++mi)
          xf[mi] = *reinterpret_cast<const bf16x8 *>(Xs + (sub ? aread1 : aread) + mi * 16 * 128);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int mi = 0; mi < WMI; ++mi)
            acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], xf[mi], acc[ni][mi], 0, 0, 0);
      }
    }
    // acc[ni][mi][j] = y[row, n0 + wc*32 + ni*16 + 4*(lane>>4) + j], row = tile + wr*32 + mi*16 + lane&15
    const int rbase = (t0 + i) * kBM + wr * 32 + (lane & 15);
#pragma unroll
    for (int mi = 0; mi < WMI; ++mi) {
      const int m = rbase + mi * 16;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[ni][mi][j] + bias4[ni][j];
          if (a.relu) v[j] = fmaxf(v[j], 0.0f);
        }
        const int64_t o = (int64_t)m * a.os + n0 + wc * 32 + ni * 16 + 4 * (lane >> 4);
        if (m < M) {
          if (a.out_f32)
            *reinterpret_cast<float4 *>(reinterpret_cast<float *>(a.out) + o) = make_float4(v[0], v[1], v[2], v[3]);
          else if (a.out_sc1)
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                   bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]}),
                __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, 0x7fffffff, 0x00020000), (uint32_t)o * 2u, 0, 16);
          else
            *reinterpret_cast<bf16x4 *>(out + o) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        }
      }
    }
    buf = buf == NA - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

}  // namespace

bool wres_launch(const WresArgs &a, int num_cus, hipStream_t s) {
  if (a.N % kBN != 0 || a.K % 64 != 0 || a.K < 64 || a.K > 256 || num_cus <= 0) return false;
  if ((a.xs & 7) || (a.os & 3)) return false;
  const int nslice = a.N / kBN;
  if (nslice > num_cus) return false;
  const int workers = num_cus / nslice;
  const dim3 grid(nslice * workers), block(512);
  WresArgs b = a;
  static const int out_sc1 = [] {  // as conv_common.h env_out_sc1: FS2_OUT_SC1=0 -> plain stores
    const char *e = getenv("FS2_OUT_SC1");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  b.out_sc1 = out_sc1;
  switch (a.K / 64) {
    case 1: hipLaunchKernelGGL(gemm_wres_kernel<1>, grid, block, 0, s, b, nslice, workers); break;
    case 2: hipLaunchKernelGGL(gemm_wres_kernel<2>, grid, block, 0, s, b, nslice, workers); break;
    case 3: hipLaunchKernelGGL(gemm_wres_kernel<3>, grid, block, 0, s, b, nslice, workers); break;
    default: hipLaunchKernelGGL(gemm_wres_kernel<4>, grid, block, 0, s, b, nslice, workers); break;
  }
  return true;
}
