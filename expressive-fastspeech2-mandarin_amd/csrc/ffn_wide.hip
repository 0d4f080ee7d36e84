// PositionwiseFeedForward + residual + LayerNorm for SMALL row counts (the encoder's B x L_max
// phoneme rows, a free-running decoder's ~10k frames) as two wide-tile launches:
//
//   launch 1 (ffn_hidden_kernel): H = relu(Conv1d_k9(x; w1) + b1)        [rows, F] bf16
//   launch 2 (ffn_out_kernel):    y = LN(H . w2^T + b2 + x) ; masked ; (+ addvecs)
//                                                        -- transformer/SubLayers.py:85-93
//
// Why: the fused kernel (ffn.hip) streams ALL 5.2 MB of FFN weights through every workgroup, which is
// right when 112-row tiles fill the chip (the cfg2 decoder's 24.9k frames) but not at 4k rows: there
// it needs 64-row tiles split 4 ways over the hidden dimension, each workgroup pulling 1.3 MB of
// weights for 64 rows at the ~70 GB/s an XCD's L2 delivers per CU (MI355X_MICROARCH.md, L2 table),
// plus a 196 KB partial hand-off: 39-42 us per encoder block at 0.21 of the MFMA peak.
//
// Launch 1 tiles 256 rows x 64 hidden columns (cfg2 encoder: 16 x 16 = 256 workgroups, one per CU):
// the x tile (256 + KS - 1 rows, all 256 channels, 144 KB) stays in LDS for all 9 taps and the
// workgroup streams only its 64-column slice of w1 (288 KB): ~0.44 MB per CU instead of ~1.5 MB. 4
// waves = 2 row halves x 2 hidden halves: a wave's k-step is 2 weight fragments (its 32 hidden rows,
// from the ffn.hip fragment-ordered image, through a register ring 8 k-steps deep), 8 B fragments
// from the x tile and 16 MFMAs; the B fragments of one row half are shared through L1-free LDS reads
// (32 KB of LDS reads and 8 KB of L1 weight reads per k-step per CU: half of either unit's rate).
//
// Launch 2 tiles 64 rows x 64 output columns (4 column quarters per row tile): K = F split over the
// 4 waves (every load of the workgroup -- 128 KB of w2, 128 KB of H -- issued at once: one memory
// round trip), the 4 partials summed in wave order through LDS, + b2 + the residual; the LayerNorm
// needs whole 256-column rows, so each quarter stores its f32 pre-norm rows (write-through) into the
// split-K workspace, and the last of the 4 to arrive (an arrival counter per row tile, as ffn.hip's
// split-hidden form) normalises all 256 columns of the tile's rows: mask, addvecs, bf16 out.
//
// Both GEMMs accumulate in the fused kernel's k order (k-steps of 32 channels, tap-major for w1,
// hidden order for w2), so H and the pre-norm sums are the fused kernel's; only the LayerNorm's row
// statistics are summed in a different order (tests/test_gpu_ffn.py: within bf16 rounding).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "conv_common.h"
#include "fs2_common.h"

#ifndef WIDE_TRACE
#define WIDE_TRACE 0  // analysis builds only: thread 0's shader clock at each phase into the workspace tail
#endif

namespace {

constexpr int kWD = 256;          // d_model
constexpr int kWUnit = 4096;      // ffn.hip weight unit: 64 rows x 32 channels, fragment order
constexpr int kWLgkm0 = 0xC07F;

template <int N, typename Fn, int... I>
__device__ __forceinline__ void wfor_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void wfor(Fn &&f) {
  wfor_impl<N>(f, std::make_integer_sequence<int, N>{});
}

struct WideArgs {
  const bf16 *x;         // FFN input rows (also the residual), row stride xs elements
  int64_t xs;
  uint32_t x_bytes;
  const bf16 *w;         // ffn.hip fragment-ordered w1 | w2 (ops.pack_ffn_weights)
  uint32_t w_bytes;
  const float *b1, *b2, *gamma, *beta;
  float eps;
  const int64_t *lens;   // padded rows: [B] lengths (mask), else null
  const float *av1, *av2;  // padded rows: [B, 256] vectors added after the mask, or null
  const int *rows_dev;   // packed rows: device row count, else null
  const int2 *row_pos;   // packed rows: (position, length) per row
  int M, T, pad, F;
  bf16 *h;               // [M, F] hidden
  uint32_t h_bytes;
  int *cnt;              // [row tiles] arrival counters (zero between launches)
  float *z;              // [M, 256] f32 pre-norm rows (split-K workspace)
  uint32_t z_bytes;
  bf16 *out;
  int64_t os;
  int nslices, ntiles;   // launch 1: hidden slices (F / 64) and 256-row tiles; launch 2: 64-row tiles
  uint64_t *trace;       // WIDE_TRACE builds: 512 workgroups x 8 stamps per launch, else null
};

// WIDE_TRACE: stamps of thread 0 (s_memtime) at the phase boundaries, written at the end
struct Stamps {
  uint64_t t[8];
  int n = 0;
  __device__ __forceinline__ void at() {
    if (WIDE_TRACE) {
      __builtin_amdgcn_sched_barrier(0);
      t[n++] = __builtin_readcyclecounter();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __device__ __forceinline__ void put(uint64_t *tr, int slot) {
    if (WIDE_TRACE && tr != nullptr && threadIdx.x == 0 && slot < 512) {
      for (int i = 0; i < n; ++i) tr[slot * 8 + i] = t[i];
      tr[slot * 8 + 7] = (uint64_t)n;
    }
  }
};

// ---------------------------------------------------------------------------------------------------
// launch 1: H = relu(conv_k(x) + b1) on 256-row x 64-column tiles
//
// The x tile (256 + KS - 1 rows x 256 channels) is STREAMED through LDS channel chunk by channel chunk
// and the k loop runs chunk-major (for each 32-channel chunk c, the KS taps): a 3-slot ring of chunks
// (chunk c + 2 is DMA'd into the slot chunk c - 1 left), so the first MFMAs wait for 1/8 of the tile
// and the workgroup needs 52 KB of LDS instead of 140 -- two workgroups per CU, one's prologue and
// H stores under the other's MFMAs (the whole-tile form's prologue took ~8-10k of ~36k cycles).
// Slot image: a 64-byte zero pad (the masked tap rows' fragment source) + 272 rows x 64 bytes; the
// 16-byte slot of channel group hi in row R is hi ^ (2 * bit 2 of R), which keeps every ds_read_b128
// lane group on 16 distinct slots for ANY row shift (the taps). The fragment addresses of all (tap,
// row block) pairs are computed once (invalid taps -> the zero pad); the ring slot is the
// instruction's immediate offset.
template <int KS>
__global__ __launch_bounds__(256, 2) void ffn_hidden_kernel(WideArgs p) {
  constexpr int BM = 256, XROWS = BM + KS - 1;
  constexpr int NPC = (XROWS + 15) / 16;  // DMA pieces (16 rows x 64 B) per chunk
  constexpr int CH = 64 + NPC * 1024;     // chunk region: zero pad + rows
  constexpr int NCH = kWD / 32;           // channel chunks (k-steps per tap)
  constexpr int PPW = (NPC + 3) / 4;      // pieces per wave per chunk (the last piece issued by every wave)
  constexpr int NSLOT = 3;                // chunk ring
  constexpr int SMEM = NSLOT * CH;
  static_assert(2 * SMEM <= 163840, "two workgroups per CU");
  static_assert(BM * 144 <= SMEM, "H staging fits in the ring");
  static_assert((NSLOT - 1) * CH < 65536, "slot offsets fit the ds_read immediate");
  constexpr int NK = KS * NCH;  // k-steps; weight unit of (tap t, chunk c) = t * NCH + c (ops.pack_ffn_weights)
  constexpr int MB = 8;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  Stamps st;
  st.at();

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rh = w & 1, hh = w >> 1;  // row half (128 rows), hidden half (32 columns) of the tile
  // XCD-aware order: consecutive L run on one XCD (blockIdx.x & 7 picks the XCD), slice-major, so an
  // XCD holds ~2 hidden slices' weights and all the x rows in its L2
  const int L = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int slice = L / p.ntiles, tile = L - slice * p.ntiles;
  if (slice >= p.nslices) return;
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M;
  const int m0 = tile * BM;
  if (m0 >= M) return;
  const int pad = p.pad, T = p.T;

  // the zero pads first: a ds_write behind the tile's LDS-DMA would wait for all of it
  if (tid < NSLOT * 4) *reinterpret_cast<float4 *>(smem + (tid >> 2) * CH + (tid & 3) * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
  // row positions of this lane's 8 row blocks and b1 of its 8 hidden columns, issued before the tile
  // (the chunk-0 wait covers them). Padded rows: position m % T of a length-T sequence; packed rows:
  // loaded over them (ALU writes after the loads into the same registers would wait for the loads)
  int2 rq[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = min(m0 + rh * 128 + mb * 16 + (lane & 15), M - 1);
    rq[mb] = make_int2(m % T, T);
  }
  if (p.row_pos != nullptr) {  // uniform branch around the whole loop: no wait between the loads
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) rq[mb] = p.row_pos[min(m0 + rh * 128 + mb * 16 + (lane & 15), M - 1)];
  }
  const int hcol0 = slice * 64 + hh * 32 + 4 * (lane >> 4);
  const float4 bb0 = *reinterpret_cast<const float4 *>(p.b1 + hcol0);
  const float4 bb1 = *reinterpret_cast<const float4 *>(p.b1 + hcol0 + 16);
  // chunk c of the x tile into ring slot c % 3: wave w issues pieces w, w + 4, ... and the last one
  // (every wave writes its identical bytes), PPW per chunk, so every wave's count is the same
  const rsrc_t sr = make_rsrc(p.x, p.x_bytes);
  const uint32_t srow = (uint32_t)p.xs * 2u;
  auto dma_chunk = [&](auto CI) {
    constexpr int c = decltype(CI)::value;
    const int ps = lane & 3;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = min(w + 4 * i, NPC - 1);
      const int R = pc * 16 + (lane >> 2);
      const int hl = ps ^ ((R >> 1) & 2);
      const int gm = m0 - pad + R;
      const bool ok = R < XROWS && gm >= 0 && gm < M;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          sr, (__attribute__((address_space(3))) void *)(smem + (c % NSLOT) * CH + 64 + pc * 1024), 16,
          ok ? (uint32_t)gm * srow + (uint32_t)(c * 64 + hl * 16) : kOOB, 0, 0, 0);
    }
  };
  dma_chunk(std::integral_constant<int, 0>{});
  dma_chunk(std::integral_constant<int, 1>{});

  // weight ring: RD k-steps ahead (k-step kk = c * KS + t reads ring slot kk % RD; the loop is fully
  // unrolled, so every slot index is static)
  constexpr int RD = 6;
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t wbase = (uint32_t)(slice * NK) * (uint32_t)kWUnit + (uint32_t)(hh * 2048 + lane * 16);
  bf16x8 pa[RD][2];
  auto load_at = [&](auto KI) {  // k-step kk's fragments into slot kk % RD
    constexpr int kk = decltype(KI)::value, c = kk / KS, t = kk % KS;
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t o = wbase + (uint32_t)(t * NCH + c) * (uint32_t)kWUnit;
    pa[kk % RD][0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, o, 0, 0));
    pa[kk % RD][1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, o + 1024, 0, 0));
    __builtin_amdgcn_sched_barrier(0);
  };
  wfor<RD>([&](auto I) { load_at(I); });
  // ring refills (2 loads each) issued by k-steps [a, b]: k-step kk refills iff kk + RD < NK
  auto refills = [](int a, int b) constexpr {
    int n = 0;
    for (int kk = a; kk <= b; ++kk) n += kk + RD < NK ? 2 : 0;
    return n;
  };

  // fragment addresses: (tap t, row block mb) -> LDS row R = rh*128 + 16 mb + r16 + t of slot 0, or
  // the zero pad when row + t - pad leaves the sequence (the rows' positions are needed: wait for
  // them); two 16-bit addresses per register (row blocks 2i, 2i + 1)
  const int r16 = lane & 15, hi = lane >> 4;
  uint32_t adp[KS][MB / 2];
  {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + 2 * RD) : "memory");  // rows + b1 (older than the tile)
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int R0 = rh * 128 + r16 + t;
      const int sl = (hi ^ ((R0 >> 1) & 2)) * 16;  // bit 2 of R is the same for every row block (16 mb)
#pragma unroll
      for (int i = 0; i < MB / 2; ++i) {
        uint32_t a2[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int mb = 2 * i + j;
          const bool ok = (unsigned)(rq[mb].x + t - pad) < (unsigned)rq[mb].y;
          a2[j] = ok ? (uint32_t)(64 + (R0 + 16 * mb) * 64 + sl) : 0u;
        }
        adp[t][i] = a2[0] | (a2[1] << 16);
      }
    }
  }
  static_assert(CH < 65536, "16-bit fragment addresses");
  // chunk c landed (this wave's pieces, then everyone's): vector-memory ops this wave issued after
  // chunk c's last piece -- chunk 0: chunk 1's pieces + the ring prologue; chunk 1: the ring prologue
  // + chunk 0's refills before its last k-step; chunk c >= 2 (issued inside the last k-step of chunk
  // c - 2, behind the barrier): that k-step's refill + chunk c - 1's refills before its last k-step
  auto wait_chunk = [&](auto CI) {
    constexpr int c = decltype(CI)::value;
    constexpr int n = c == 0 ? PPW + 2 * RD
                             : c == 1 ? 2 * RD + refills(0, KS - 2)
                                      : refills((c - 2) * KS + KS - 1, (c - 1) * KS + KS - 2);
    static_assert(n <= 63, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
    __builtin_amdgcn_s_waitcnt(kWLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  wait_chunk(std::integral_constant<int, 0>{});
  st.at();

  f32x4 acc[2][MB];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](auto CI, auto TI, bf16x8 (&f)[MB]) {
    constexpr int c = decltype(CI)::value, t = decltype(TI)::value, off = (c % NSLOT) * CH;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      // volatile: unpacked per use (hipcc would otherwise keep all 72 unpacked addresses live across
      // the unrolled chunks and spill)
      uint32_t a;
      asm volatile("v_bfe_u32 %0, %1, %2, 16" : "=v"(a) : "v"(adp[t][mb >> 1]), "n"((mb & 1) * 16));
      f[mb] = *reinterpret_cast<const bf16x8 *>(smem + a + off);
    }
  };
  auto mma = [&](const bf16x8 (&fa)[2], const bf16x8 (&fb)[MB]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[jb], fb[mb], acc[jb][mb], 0, 0, 0);
  };
  bf16x8 f0[MB], f1[MB];
  issue(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, f0);
  wfor<NCH>([&](auto CI) {
    constexpr int c = decltype(CI)::value;
    wfor<KS>([&](auto TI) {
      constexpr int t = decltype(TI)::value;
      constexpr int kk = c * KS + t;  // k-step index: f0 / f1 alternate
      // next k-step's fragments first (one k-step of LDS latency hidden under this one's MFMAs)
      if constexpr (t + 1 < KS) {
        if constexpr (kk & 1)
          issue(CI, std::integral_constant<int, t + 1>{}, f0);
        else
          issue(CI, std::integral_constant<int, t + 1>{}, f1);
      } else if constexpr (c + 1 < NCH) {
        wait_chunk(std::integral_constant<int, c + 1>{});
        // every wave is past chunk c - 1: its slot takes chunk c + 2
        if constexpr (c + 2 < NCH) dma_chunk(std::integral_constant<int, c + 2>{});
        if constexpr (kk & 1)
          issue(std::integral_constant<int, c + 1>{}, std::integral_constant<int, 0>{}, f0);
        else
          issue(std::integral_constant<int, c + 1>{}, std::integral_constant<int, 0>{}, f1);
      }
      if constexpr (kk & 1)
        mma(pa[kk % RD], f1);
      else
        mma(pa[kk % RD], f0);
      if constexpr (kk + RD < NK) load_at(std::integral_constant<int, kk + RD>{});
    });
  });
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __builtin_amdgcn_s_barrier();  // every wave done with the x tile: stage H over it
  st.at();

  // H = bf16(relu(acc + b1)): lane holds hidden columns 4 hi .. +3 of block jb, row hrow0 + 16 mb;
  // staged at a 144-byte row pitch, then whole 128-byte row segments out (8 x 16 B per row)
  constexpr int HP = 144;
  const int hrow0 = rh * 128 + r16;
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const float4 bb = jb == 0 ? bb0 : bb1;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 v = acc[jb][mb];
      bf16x4 o;
      o[0] = (bf16)fmaxf(v[0] + bb.x, 0.f);
      o[1] = (bf16)fmaxf(v[1] + bb.y, 0.f);
      o[2] = (bf16)fmaxf(v[2] + bb.z, 0.f);
      o[3] = (bf16)fmaxf(v[3] + bb.w, 0.f);
      *reinterpret_cast<bf16x4 *>(smem + (hrow0 + 16 * mb) * HP + (hh * 32 + jb * 16 + 4 * hi) * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __syncthreads();
  const uint32_t hrow = (uint32_t)p.F * 2u;
  char *hb = reinterpret_cast<char *>(p.h);
#pragma unroll
  for (int i = 0; i < BM * 8 / 256; ++i) {
    const int e = tid + 256 * i, r = e >> 3, c = e & 7;
    if (m0 + r < M)
      *reinterpret_cast<uint4 *>(hb + (uint32_t)(m0 + r) * hrow + (uint32_t)(slice * 128 + c * 16)) =
          *reinterpret_cast<const uint4 *>(smem + r * HP + c * 16);
  }
  if (WIDE_TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st.at();
    st.put(p.trace, L);
  }
}

// ---------------------------------------------------------------------------------------------------
// launch 2: z = H . w2^T + b2 + x on 64-row x 64-column tiles, then the LayerNorm by the last of the
// row tile's 4 column quarters
template <int F>
__global__ __launch_bounds__(256, 1) void ffn_out_kernel(WideArgs p) {
  constexpr int NK = F / 32;       // k-steps of 32 hidden columns
  constexpr int KW = NK / 4;       // per wave
  constexpr int RED = 4 * 16 * 64 * 16;  // 4 waves' partial tiles in LDS: [wave][jb * 4 + mb][lane] f32x4
  constexpr int VEC = RED;               // gamma | beta (f32, by LDS-DMA at kernel start)
  constexpr int OP = kWD * 2 + 16;       // LayerNorm output staging pitch (over the partials)
  static_assert(64 * OP <= RED, "staging fits");
  __shared__ __attribute__((aligned(16))) char smem[RED + 2048 + 16];
  Stamps st;
  st.at();

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the 4 quarters of a row tile adjacent in L (one XCD: the hand-off stays in its L2)
  const int L = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int tile = L >> 2, q = L & 3;
  if (tile >= p.ntiles) return;
  const int M = p.rows_dev != nullptr ? min(*p.rows_dev, p.M) : p.M;
  const int m0 = tile * 64;
  if (m0 >= M) return;
  const int T = p.T;
  const int hi = lane >> 4, r16 = lane & 15;
  // the LayerNorm vectors into LDS first (only the last arriver reads them, after its vmcnt(0))
  if (w < 2)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(w == 0 ? p.gamma : p.beta, 1024),
                                             (__attribute__((address_space(3))) void *)(smem + VEC + w * 1024), 16,
                                             (uint32_t)lane * 16u, 0, 0, 0);

  // every operand of this wave's K quarter at once: KW k-steps x (4 w2 fragments + 4 H fragments)
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const rsrc_t hr = make_rsrc(p.h, p.h_bytes);
  bf16x8 wa[KW][4], hb[KW][4];
  // w2 units after w1 (the last kWD * F elements of the image): quarter q's k-step kk at unit q * NK + kk
  const uint32_t wb = p.w_bytes - (uint32_t)(kWD * F * 2) + (uint32_t)((q * NK + w * KW) * kWUnit) + (uint32_t)lane * 16u;
  const uint32_t hrow = (uint32_t)F * 2u;
#pragma unroll
  for (int k = 0; k < KW; ++k) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
      wa[k][jb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, wb + k * kWUnit + jb * 1024, 0, 0));
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m = m0 + mb * 16 + r16;
      hb[k][mb] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      hr, m < M ? (uint32_t)m * hrow + (uint32_t)((w * KW + k) * 64 + hi * 16) : kOOB, 0, 0));
    }
  }
  // + b2 + residual operands of this lane (row m0 + 16 w + r16, columns 64 q + 16 jb + 4 hi .. + 3),
  // loaded with the rest: a load issued after the first z store would wait for that store
  const int m = m0 + 16 * w + r16;
  const bool mok = m < M;
  const rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const rsrc_t zr = make_rsrc(p.z, p.z_bytes);
  float4 b2v[4];
  uint2 xv[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int n = 64 * q + 16 * jb + 4 * hi;
    b2v[jb] = *reinterpret_cast<const float4 *>(p.b2 + n);
    xv[jb] = bload8(xr, mok ? (uint32_t)m * (uint32_t)p.xs * 2u + (uint32_t)n * 2u : kOOB);
  }
  // all loads stay ahead of the MFMAs (left alone, hipcc interleaves them to save registers and
  // every k-step then waits for its own memory round trip)
  __builtin_amdgcn_sched_barrier(0);
  if (WIDE_TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st.at();
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KW; ++k)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[k][jb], hb[k][mb], acc[jb][mb], 0, 0, 0);
  // the 4 K-quarter partials through LDS, summed in wave order by the wave owning row block mb = w
  f32x4 *red = reinterpret_cast<f32x4 *>(smem);
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) red[(w * 16 + jb * 4 + mb) * 64 + lane] = acc[jb][mb];
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __builtin_amdgcn_s_barrier();
  st.at();
  f32x4 zv[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    f32x4 s = red[(0 * 16 + jb * 4 + w) * 64 + lane];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) s += red[(ww * 16 + jb * 4 + w) * 64 + lane];
    zv[jb] = s;
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int n = 64 * q + 16 * jb + 4 * hi;
    const bf16x4 x4 = __builtin_bit_cast(bf16x4, xv[jb]);
    f32x4 v = zv[jb];
    v[0] = v[0] + b2v[jb].x + (float)x4[0];
    v[1] = v[1] + b2v[jb].y + (float)x4[1];
    v[2] = v[2] + b2v[jb].z + (float)x4[2];
    v[3] = v[3] + b2v[jb].w + (float)x4[3];
    // write-through (sc1): the last-arriving quarter reads it with sc1 loads from another CU
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), zr,
                                           mok ? ((uint32_t)m * kWD + (uint32_t)n) * 4u : kOOB, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  st.at();
  int *flag = reinterpret_cast<int *>(smem + RED + 2048);
  if (tid == 0) {
    // relaxed add + sc1 stores / loads of every handed-off byte, each storing wave drained before the
    // barrier ahead of this add, one workgroup per CU: ffn.hip's split-hidden hand-off
    const int old = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == 3;
    if (last) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    *flag = last;
  }
  __syncthreads();
  st.at();
  if (!*flag) {
    st.put(p.trace, L);
    return;
  }

  // LayerNorm of the tile's rows over all 256 columns: wave w takes rows 16 w + r16; lane (r16, hi)
  // holds columns 16 i + 4 hi .. + 3, i = 0..15 (64 values); row sums over the 4 lanes of a row.
  // The bf16 rows are staged in LDS (over the partials) and leave as whole 512-byte rows.
  if (mok) {
    f32x4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           zr, ((uint32_t)m * kWD + (uint32_t)(16 * i + 4 * hi)) * 4u, 0, 16));
    bool masked = false;
    int bb = 0;
    if (p.row_pos == nullptr) {
      bb = m / T;
      masked = p.lens != nullptr && (int64_t)(m - bb * T) >= p.lens[bb];
    }
    float4 a1[16], a2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = 16 * i + 4 * hi;
      a1[i] = p.av1 != nullptr ? *reinterpret_cast<const float4 *>(p.av1 + (int64_t)bb * kWD + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.0f / 256.0f);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      v[i] -= mean;
      ss += (v[i][0] * v[i][0] + v[i][1] * v[i][1]) + (v[i][2] * v[i][2] + v[i][3] * v[i][3]);
    }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = 1.0f / sqrtf(ss * (1.0f / 256.0f) + p.eps);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = 16 * i + 4 * hi;
      a2[i] = p.av2 != nullptr ? *reinterpret_cast<const float4 *>(p.av2 + (int64_t)bb * kWD + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float *vg = reinterpret_cast<const float *>(smem + VEC), *vb = vg + kWD;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = 16 * i + 4 * hi;
      const float4 g = *reinterpret_cast<const float4 *>(vg + n);
      const float4 be = *reinterpret_cast<const float4 *>(vb + n);
      float y[4] = {v[i][0] * rstd * g.x + be.x, v[i][1] * rstd * g.y + be.y, v[i][2] * rstd * g.z + be.z,
                    v[i][3] * rstd * g.w + be.w};
      if (masked) y[0] = y[1] = y[2] = y[3] = 0.f;
      // addvecs after the mask, every row
      if (p.av1 != nullptr) {
        y[0] += a1[i].x; y[1] += a1[i].y; y[2] += a1[i].z; y[3] += a1[i].w;
      }
      if (p.av2 != nullptr) {
        y[0] += a2[i].x; y[1] += a2[i].y; y[2] += a2[i].z; y[3] += a2[i].w;
      }
      const bf16x4 o = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
      *reinterpret_cast<bf16x4 *>(smem + (16 * w + r16) * OP + n * 2) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(kWLgkm0);
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + 256 * i, r = e >> 5, c = e & 31;
    if (m0 + r < M)
      *reinterpret_cast<uint4 *>(p.out + (int64_t)(m0 + r) * p.os + c * 8) =
          *reinterpret_cast<const uint4 *>(smem + r * OP + c * 16);
  }
  if (WIDE_TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st.at();
    st.put(p.trace, L);
  }
}

}  // namespace

extern "C" int fs2_ffn_wide(const fs2_ffn_desc *d, void *hidden, int64_t hidden_bytes, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->b1 == nullptr || d->b2 == nullptr ||
      d->ln_gamma == nullptr || d->ln_beta == nullptr || d->out == nullptr || hidden == nullptr)
    return FS2_EINVAL;
  if (d->B < 0 || d->T < 0 || d->x_row_stride < kWD || (d->x_row_stride & 7) || d->out_row_stride < kWD ||
      (d->out_row_stride & 7))
    return FS2_EINVAL;
  if (d->D != kWD || !(d->F == 1024 || d->F == 512) || !(d->KS == 9 || d->KS == 3) || d->pad < 0 ||
      d->pad > d->KS - 1)
    return FS2_EUNSUPPORTED;
  if (d->wqkv != nullptr || d->pre_att != nullptr) return FS2_EUNSUPPORTED;  // fused-kernel extras
  if ((d->rows_dev == nullptr) != (d->row_pos == nullptr)) return FS2_EINVAL;
  if (d->rows_dev != nullptr && (d->lens != nullptr || d->addvec1 != nullptr || d->addvec2 != nullptr))
    return FS2_EINVAL;
  if (d->x == d->out || hidden == d->x || hidden == d->out) return FS2_EINVAL;
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 > 0x7fffff00LL || d->rows_max < 0) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;
  const int64_t Mg = (d->rows_dev != nullptr && d->rows_max > 0 && d->rows_max < M64) ? d->rows_max : M64;
  const int64_t xb = M64 * d->x_row_stride * 2;
  const int64_t wb = ((int64_t)d->F * d->KS * kWD + (int64_t)kWD * d->F) * 2;  // ffn.hip: w1 | w2
  const int64_t hb = Mg * d->F * 2;
  const int ntiles64 = (int)((Mg + 63) / 64);
  const int64_t zb = Mg * kWD * 4;
  if (xb >= (1LL << 31) || hb >= (1LL << 31) || hidden_bytes < hb) return FS2_EUNSUPPORTED;
  if (d->splitk_ws == nullptr || ntiles64 > 1024 || d->splitk_ws_bytes < 4096 + zb || zb >= (1LL << 31))
    return FS2_EINVAL;
  WideArgs p{};
  p.x = reinterpret_cast<const bf16 *>(d->x);
  p.xs = d->x_row_stride;
  p.x_bytes = (uint32_t)xb;
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.w_bytes = (uint32_t)wb;
  p.b1 = d->b1;
  p.b2 = d->b2;
  p.gamma = d->ln_gamma;
  p.beta = d->ln_beta;
  p.eps = d->ln_eps;
  p.lens = d->lens;
  p.av1 = d->addvec1;
  p.av2 = d->addvec2;
  p.rows_dev = d->rows_dev;
  p.row_pos = reinterpret_cast<const int2 *>(d->row_pos);
  p.M = (int)Mg;
  p.T = d->T;
  p.pad = d->pad;
  p.F = d->F;
  p.h = static_cast<bf16 *>(hidden);
  p.h_bytes = (uint32_t)hb;
  p.cnt = static_cast<int *>(d->splitk_ws);
  p.z = reinterpret_cast<float *>(static_cast<char *>(d->splitk_ws) + 4096);
  p.z_bytes = (uint32_t)zb;
  p.out = static_cast<bf16 *>(d->out);
  p.os = d->out_row_stride;
  if (WIDE_TRACE)
    p.trace = reinterpret_cast<uint64_t *>(static_cast<char *>(d->splitk_ws) + d->splitk_ws_bytes - 65536);
  hipStream_t s = as_stream(stream);
  // launch 1: hidden slices x 256-row tiles, grid padded to whole XCD rounds
  p.nslices = d->F / 64;
  p.ntiles = (int)((Mg + 255) / 256);
  const int n1 = (p.nslices * p.ntiles + 7) & ~7;
  // launch 1 fits twice per CU (LDS, registers): two co-resident workgroups overlap one's prologue
  // and H stores with the other's MFMAs (free-running decoder rows: 656 workgroups); with at most one
  // workgroup per CU to launch, extra dynamic LDS keeps it at one per CU
  constexpr int kCUs = 256;
  // (static LDS 52 KB; + 32 KB is past half of the CU's 160 KB)
  const size_t solo = 32 * 1024;
  if (d->KS == 9)
    hipLaunchKernelGGL((ffn_hidden_kernel<9>), dim3(n1), dim3(256), n1 <= kCUs ? solo : 0, s, p);
  else
    hipLaunchKernelGGL((ffn_hidden_kernel<3>), dim3(n1), dim3(256), n1 <= kCUs ? solo : 0, s, p);
  FS2_CHECK_LAUNCH();
  // launch 2: 64-row tiles x 4 column quarters
  p.ntiles = ntiles64;
  if (WIDE_TRACE) p.trace += 4096;
  const int n2 = (ntiles64 * 4 + 7) & ~7;
  if (d->F == 1024)
    hipLaunchKernelGGL((ffn_out_kernel<1024>), dim3(n2), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((ffn_out_kernel<512>), dim3(n2), dim3(256), 0, s, p);
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}
