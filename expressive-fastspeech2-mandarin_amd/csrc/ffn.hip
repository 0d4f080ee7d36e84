// PositionwiseFeedForward + residual + LayerNorm + padding mask as ONE kernel (gfx950 / CDNA4):
//
//   f = relu(Conv1d_k9(x; w1) + b1)              [rows, 1024]   -- never leaves the CU
//   y = LN(f . w2^T + b2 + x) ; masked ; (+ addvec)               -- transformer/SubLayers.py:85-93
//
// Why one kernel: as two launches the 1024-wide hidden f is written to HBM by the k=9 conv and
// read back by the k=1 conv (cfg2 decoder: 51 MB each way per block), and the k=1 conv + LN runs
// as its own latency-bound launch (18 % of MFMA peak). Here a workgroup owns BM = 112 rows for
// the whole FFN and walks the hidden dimension in chunks of 256 columns:
//
//   for chunk c:  GEMM1  H^T[j, m] = sum_{tap, ch} W1[c*256 + j, tap, ch] . X[m + tap - pad, ch]
//                 H = relu(H^T + b1) -> bf16 -> LDS [112 x 256]            (chunk of f, on chip)
//                 GEMM2  Y^T[n, m] += sum_j W2[n, c*256 + j] . H[m, j]      (accumulated in registers)
//   LN epilogue on Y (through LDS, conv_common.h's epilogue).
//
// Both GEMMs put the WEIGHTS on the MFMA A side (rows j / n, 16 per block) and the activations on
// the B side (columns m). 4 waves, one per SIMD, 512 registers each: wave w owns weight rows
// 64w .. 64w+63 of every k-step and all 112 activation rows, so its two accumulators (H^T and
// Y^T, 4 x 7 blocks of 16x16 f32 each) sit in the accumulator registers for the whole kernel.
//
// Data movement. A wave's weight rows are its own (no other wave reads them), so they never touch
// LDS: the packed buffer (ops.pack_ffn_weights) stores each wave k-step ("unit": 64 rows x 32
// channels, 28 MFMAs) as 4 KiB in fragment order, loaded by 4 fully coalesced 16-byte-per-lane
// buffer loads straight into A-operand registers, DEPTH units ahead (a register ring). The
// activations are shared: the x tile with the taps' halo (BM + KS - 1 rows x 512 B) is DMA'd to
// LDS once, and each unit reads its 7 B fragments (rows shifted by the tap) one unit ahead of its
// MFMAs. GEMM1 needs no barrier at all; two per chunk hand the hidden slice H over. LDS holds the
// x tile (60 KiB), H (56 KiB) and b1; the LN epilogue reuses it. A fragment whose shifted row
// leaves its sequence reads a 16-byte zero slot instead (address select, no branch).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

#ifndef FFN_TRACE
#define FFN_TRACE 0  // analysis builds only: per-phase shader-clock stamps of wave 0 into spare output rows
#endif
#ifndef FFN_ABLATE
#define FFN_ABLATE 0  // analysis builds only: bit 0 no MFMAs, bit 1 no weight loads, bit 2 no B-fragment reads, bit 3 every
                      // weight load reads unit 0 (L1-resident), bit 4 no tap masking
#endif

constexpr int kD = 256;            // d_model (encoder_hidden / decoder_hidden)
constexpr int kChunk = 256;        // hidden columns per chunk
constexpr int kUnit = 4096;        // bytes of one wave unit: 4 row blocks x 64 lanes x 16 B
constexpr int kDepth = 4;          // weight units in flight per wave (register ring)

struct FfnArgs {
  ConvArgs e;          // x / rows / LN epilogue fields (conv_common.h); e.w unused
  const bf16 *w;       // fs2_ffn_desc.w: w_1 | w_2 in fragment order (include/fs2hip.h)
  const float *b1;     // [F]
  uint32_t w_bytes;
  int nsplit;          // split-hidden form: workgroups per row tile (1 = off)
  int ntiles;          // row tiles of the launch
  int *cnt;            // [tiles] arrival counters (zero between launches)
  void *part;          // f32 partial Y^T accumulators, part_bytes(MB) per (tile, split)
  int acquire;         // agent acquire before the partial loads (FS2_FFN_ACQUIRE=1; off: sc1 hand-off)
  int out_sc1;         // output rows stored write-through (sc1): the lines leave L2 (FS2_OUT_SC1=0: plain, A/B)
  int prefetch;        // split-hidden form: L2 warm-up of the split's weights (FS2_FFN_PREFETCH)
  uint32_t part_bytes;
  // the NEXT FFT block's Q|K|V projection of y (optional): qkv[m, :] = y[m, :] . wq^T + bq
  const bf16 *wq;      // [nq][256] in fragment order [nq/64][8][4][4][16][8]
  const float *bq;     // [nq]
  bf16 *qkv;           // [rows, >= nq]
  int64_t qs;          // qkv row stride (elements)
  uint32_t wq_bytes;
  int nq;              // multiple of 256
  // the block's attention output projection + residual + LayerNorm in the prologue (PRE kernels):
  // the FFN input h = LN1(att . wfc^T + bfc + x) of the tile and its halo rows, computed on chip
  const bf16 *att;     // [rows, >= 256]
  int64_t as;
  uint32_t att_bytes;
  const bf16 *wfc;     // [256][256] in fragment order [4][8][4][4][16][8]
  const float *bfc, *g1, *be1;
  float eps1;
};

// f32 partial Y^T accumulators per (tile, split): 4 waves x acc2[4][MB] x 64 lanes x 16 B
constexpr int part_bytes(int MB) { return 4 * 4 * MB * 64 * 16; }

constexpr int64_t ffn_weight_elems(int KS, int F) { return (int64_t)F * KS * kD + (int64_t)kD * F; }

// physical 16-byte chunk of logical chunk c in a 512-byte LDS row r: ds_read_b128 of 16
// consecutive rows starting anywhere (the tap shift) conflict-free, and the 8-byte accesses of one
// column across 16 rows (H writes, residual reads, output staging) 2-way -- the least possible for
// that pattern (the swizzle `(r & 7) << 1` made them 4-way). Found by exhaustive search over XOR
// maps of the row bits; depends on r & 7 only.
__device__ __forceinline__ int xchunk(int r, int c) { return c ^ ((r & 3) << 1) ^ ((r & 4) ? 9 : 0); }

template <int N, typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

// lgkmcnt(0) as a real s_waitcnt the compiler's wait-count pass sees: gfx9 simm16 = vmcnt 63
// (bits 3:0 and 15:14), expcnt 7, lgkmcnt 0
constexpr int kLgkm0 = 0xC07F;
// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 encoding: vmcnt [3:0] + [15:14])
constexpr int vm_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

// MB = 16-row activation blocks per tile: 7 (112 rows: the full-chip decoder launches), 6 (96 rows x 2
// hidden splits: a free-running decoder's ~8-12k rows, 232 workgroups that stream half the weights
// each) or 4 (64 rows: the split-hidden form of small launches, whose 4 splits x 64-row tiles fill the chip)
template <int KS, int NCH, int MB, bool PRE = false>
__global__ __launch_bounds__(256, 1) void ffn_fused_kernel(FfnArgs p) {
  constexpr int BM = 16 * MB;
  constexpr uint32_t kPartBytes = (uint32_t)part_bytes(MB);
  constexpr int XROWS = BM + KS - 1;
  // x tile rows at a 544-byte pitch (512 + 32): the 16 rows of a fragment read fall in 16 distinct
  // bank groups for any tap shift with NO swizzle, so a unit's k-step is a constant byte offset
  // (the ds_read immediate) and the per-unit address work disappears
  constexpr int XPITCH = 544;
  constexpr int XPIECES = (XROWS * XPITCH + 1023) / 1024;  // 1 KiB LDS-DMA pieces
  constexpr int XP_PER_WAVE = (XPIECES + 3) / 4;
  // a 512-byte zero region at LDS offset 0: a masked row's fragment address is (address & 0) plus
  // the k-step offset, which stays inside it
  constexpr int ZERO_OFF = 0;
  constexpr int X_OFF = 512;
  constexpr int H_OFF = X_OFF + 4 * XP_PER_WAVE * 1024;
  constexpr int F = NCH * kChunk;
  constexpr int B1_OFF = H_OFF + BM * 512;
  constexpr int EP_OFF = B1_OFF + F * 4;            // b2, gamma, beta: 3 x 256 f32
  constexpr int RED_OFF = EP_OFF + 3 * kD * 4;      // LN row statistics: [BM rows][4 waves] f32
  // PRE: the attention-output tile (XROWS rows at the x pitch) over the H / vector regions, and
  // its LN row statistics after it; both dead before GEMM1 starts
  constexpr int ATT_OFF = H_OFF;
  constexpr int RED0_OFF = ATT_OFF + 4 * XP_PER_WAVE * 1024;
  constexpr int SMEM0 = RED_OFF + BM * 16;
  constexpr int VEC0_OFF = RED0_OFF + 64 * 16;   // PRE: bfc, gamma1, beta1 (3 x 256 f32)
  constexpr int SMEM = PRE && VEC0_OFF + 3 * kD * 4 > SMEM0 ? VEC0_OFF + 3 * kD * 4 : SMEM0;
  static_assert(SMEM <= 163840, "LDS");
  static_assert(BM * 528 <= 4 * XP_PER_WAVE * 1024, "Q|K|V staging fits in the x region");
  constexpr int NK1 = KS * (kD / 32);  // GEMM1 units per chunk (tap-major, 8 k-steps per tap)
  constexpr int NK2 = kChunk / 32;     // GEMM2 units per chunk
  constexpr int DEPTH = kDepth;
  static_assert(NK1 % DEPTH == 0 && NK2 % DEPTH == 0, "static register-ring slots");
  constexpr int SCR_OFF = SMEM + (FFN_TRACE ? 256 : 0);  // L2 warm-up scratch (1 KiB per wave), !PRE only
  __shared__ __attribute__((aligned(16))) char smem[SCR_OFF + (PRE ? 0 : 4096)];

  const ConvArgs &a = p.e;
  const uint64_t t_entry = FFN_TRACE ? __builtin_readcyclecounter() : 0;  // trace builds: kernel entry
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // weight-row quarter (64 rows)
  const int M = a.rows_dev != nullptr ? min(*a.rows_dev, a.M) : a.M;
  // split-hidden form: the grid (a multiple of 8) walks (split, tile) split-major and XCD-major, so
  // an XCD runs (mostly) ONE split and its L2 holds only that split's 1.3 MB of weights (tile-major
  // order puts all 5.2 MB through every 4 MB L2; measured equal at the encoder shape, where the
  // partial hand-off, not the weight stream, is what the split form pays for)
  const int S = p.nsplit;
  int tile = blockIdx.x, split = 0;
  if (S > 1) {
    const int ntiles = p.ntiles;
    const int L = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    split = L / ntiles;
    tile = L - split * ntiles;
    if (split >= S) return;
  }
  const int m0 = tile * BM;
  if (m0 >= M) return;
  const int nchunks = NCH / S, c0 = split * nchunks, cend = c0 + nchunks;
  const int pad = a.pad, T = a.T;

  // ---- tap validity of this lane's activation rows: bit tap of vmask[mb] is set when the row
  // shifted by tap - pad stays inside its sequence (sequence position / length)
  int vmask[MB];
  // padded rows with lengths: bit mb set when this lane's row of block mb is padding (t >= lens[b]),
  // read here, beside the x tile DMA, rather than in the LN epilogue's dependent chain
  int padmask = 0;
  // every block's row_pos / lens entry is loaded before any is used (clamped row, no branch), so
  // the MB loads overlap: a per-block load + wait chain cost ~15k cycles at kernel start
  int2 rq[MB];
  int64_t rl[MB];
  if (a.row_pos != nullptr) {  // (uniform branches around whole loops: no wait between the loads)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) rq[mb] = a.row_pos[min(m0 + mb * 16 + (lane & 15), M - 1)];
  } else {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = min(m0 + mb * 16 + (lane & 15), M - 1);
      rq[mb] = make_int2(m % T, T);
    }
    if (a.lens != nullptr) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) rl[mb] = a.lens[min(m0 + mb * 16 + (lane & 15), M - 1) / T];
    } else {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) rl[mb] = T;
    }
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + mb * 16 + (lane & 15);
    int tpos = 0, tlen = 0;  // rows past M: never valid (not stored)
    if (m < M) {
      tpos = rq[mb].x;
      tlen = rq[mb].y;
      if (a.row_pos == nullptr && (int64_t)tpos >= rl[mb]) padmask |= 1 << mb;
    }
    int v = 0;
#pragma unroll
    for (int tap = 0; tap < KS; ++tap) v |= ((unsigned)(tpos + tap - pad) < (unsigned)tlen ? 1 : 0) << tap;
    vmask[mb] = v;
  }
  // 1 KiB of an f32 vector straight into LDS (LDS-DMA: no register round trip, so no wait here;
  // the vmcnt waits that cover the tiles cover these older loads too)
  auto vec_dma = [&](const float *src, int piece, char *dst) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(src, (uint32_t)(piece + 1) * 1024u),
                                             (__attribute__((address_space(3))) void *)dst, 16,
                                             (uint32_t)piece * 1024u + (uint32_t)lane * 16u, 0, 0, 0);
  };
  auto load_vectors = [&]() {
    // b1 -> LDS (F / 256 pieces over the waves); the LN epilogue's b2 / gamma / beta (waves 0-2)
    for (int pc = w; pc < F / 256; pc += 4) vec_dma(p.b1, pc, smem + B1_OFF + pc * 1024);
    if (w < 3) vec_dma(w == 0 ? a.bias : w == 1 ? a.gamma : a.beta, 0, smem + EP_OFF + w * 1024);
  };
  if constexpr (!PRE) load_vectors();
  if (tid < 32) *reinterpret_cast<float4 *>(smem + ZERO_OFF + 16 * tid) = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) asm volatile("" ::"v"(vmask[mb]));

  // trace builds: wave 0 stamps the shader clock into an LDS slot past the kernel's own LDS
  auto stamp = [&](int i) {
    if (FFN_TRACE) {
      __builtin_amdgcn_sched_barrier(0);
      const uint64_t t = __builtin_readcyclecounter();
      if (tid == 0) *reinterpret_cast<uint64_t *>(smem + SMEM + 8 * i) = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  // lane-linear 1 KiB LDS-DMA pieces of a [XROWS x 512 B] row tile at the 544-byte pitch
  auto tile_dma_range = [&](const void *src, uint32_t bytes, int64_t stride, int off, int i0, int i1) {
    const rsrc_t sr = make_rsrc(src, bytes);
    const uint32_t srow = (uint32_t)stride * 2u;
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int pc = w + 4 * i;
      const int o = pc * 1024 + lane * 16;  // lane-linear LDS image: row o / XPITCH, byte o % XPITCH
      const int r = o / XPITCH, within = o - r * XPITCH;
      const int gm = m0 - pad + r;
      const bool ok = r < XROWS && within < 512 && gm >= 0 && gm < M;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          sr, (__attribute__((address_space(3))) void *)(smem + off + pc * 1024), 16,
          ok ? (uint32_t)gm * srow + (uint32_t)within : kOOB, 0, 0, 0);
    }
  };
  auto tile_dma = [&](const void *src, uint32_t bytes, int64_t stride, int off) {
    tile_dma_range(src, bytes, stride, off, 0, XP_PER_WAVE);
  };
  // ---- weight units: register ring of DEPTH units. Every load site is static (its unit is known
  // from its position in the unrolled code), so the stream needs no branch: a branch there splits
  // the MFMA sequence and hipcc then copies the accumulators between blocks.
  constexpr uint32_t W2_BASE = (uint32_t)(F * KS * kD * 2);
  const uint32_t lane_off = (uint32_t)lane * 16u;
  auto base1 = [&](int c) { return (uint32_t)((c * 4 + w) * NK1) * (uint32_t)kUnit; };
  auto base2 = [&](int c) { return W2_BASE + (uint32_t)(w * (F / 32) + c * NK2) * (uint32_t)kUnit; };
  bf16x8 pa[DEPTH][4];
  auto load_at = [&](auto S, uint32_t so) {
    constexpr int s = decltype(S)::value;
    if (FFN_ABLATE & 2) return;
    // pinned after the MFMAs that read the slot's previous unit: a load hoisted above them keeps
    // both units live, and the register allocator then rotates the whole ring through copies
    // (each copy waiting for its load) at the loop back-edge
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, lane_off + jb * 1024, (FFN_ABLATE & 8) ? 0u : so, 0);
      pa[s][jb] = __builtin_bit_cast(bf16x8, v);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto ring_start = [&]() {
    static_for<DEPTH>([&](auto I) { load_at(I, base1(c0) + (uint32_t)(decltype(I)::value * kUnit)); });
  };
  // the first DEPTH units follow the x tile DMA (PRE: the prologue), so that the counted wait below
  // (all but the ring's 4 * DEPTH youngest loads) covers the tile
  if constexpr (!PRE) {
    // ---- split-hidden form: L2 warm-up (as vp.hip). An XCD's workgroups run ONE split (the
    // split-major order above) and stream its ~1.3 MB of weights in lockstep, 16 MFMAs per 4 KiB
    // unit at 64-row tiles: too little work to cover an XCD-wide first-touch miss with a 4-unit ring.
    // Each wave first pulls disjoint 1 KiB slices of the split's GEMM1 block and its four GEMM2
    // column ranges into a scratch slot (waited for with the x tile), so the rings then hit L2.
    if (S > 1 && p.prefetch) {
      const int nch = cend - c0;
      const int p1 = nch * 4 * NK1 * 4, p2q = nch * NK2 * 4;  // 1 KiB pieces: GEMM1 block, one GEMM2 range
      const uint32_t g1 = (uint32_t)(c0 * 4 * NK1) * (uint32_t)kUnit;
      constexpr uint32_t W2B = (uint32_t)(F * KS * kD * 2);
      const int per_xcd = (int)(gridDim.x >> 3);
      const int me = (int)(blockIdx.x >> 3) * 4 + w, nw = per_xcd * 4;
      for (int i = 0, pc = me; i < 16 && pc < p1 + 4 * p2q; ++i, pc += nw) {
        uint32_t off;
        if (pc < p1) {
          off = g1 + (uint32_t)pc * 1024u;
        } else {
          const int j = pc - p1, ww = j / p2q, r = j - ww * p2q;
          off = W2B + (uint32_t)(ww * (F / 32) + c0 * NK2) * (uint32_t)kUnit + (uint32_t)r * 1024u;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(smem + SCR_OFF + w * 1024),
                                                 16, off + (uint32_t)lane * 16u, 0, 0, 0);
      }
    }
    // ---- x tile (rows m0 - pad .. m0 + BM + KS - 2, all 256 channels) -> LDS, once
    tile_dma(a.x, a.x_bytes, a.xs, X_OFF);
    ring_start();
  } else {
    // ---- prologue GEMM0 (SubLayers.py:54-55 + Layers.py:25: fc + residual + LayerNorm): the FFN
    // input h of the tile's XROWS rows (halo included: the taps of GEMM1 read them), written as
    // the x tile. fc^T[n, m] = sum_d Wfc[n, d] att[m, d]: the 8 weight k-steps of this wave's 64
    // output channels stay in registers for both row passes (4 blocks = 64 rows each); the att
    // tile is DMA'd to LDS at the x pitch; residual rows from global; LN statistics via LDS.
    // both tiles by LDS-DMA at once: att at ATT_OFF, the block input x (the residual) at X_OFF,
    // where each lane overwrites its own elements with h (nothing else reads x in the prologue)
    // issue order: the LN vectors (oldest: their LDS store waits only for them), the fc weights,
    // then both tiles' first PRE_SPLIT pieces per wave (rows 0 .. ~67: row pass 0), then the rest --
    // pass 0 starts when its rows have landed while the second half still streams in
    const int hr = lane & 15, hq = lane >> 4;
    if (w < 3) vec_dma(w == 0 ? p.bfc : w == 1 ? p.g1 : p.be1, 0, smem + VEC0_OFF + w * 1024);
    const rsrc_t fr = make_rsrc(p.wfc, (uint32_t)(kD * kD * 2));
    const uint32_t lane_o = (uint32_t)lane * 16u;
    bf16x8 wf[8][4];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        wf[ks][jb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    fr, lane_o + (uint32_t)(jb * 1024), (uint32_t)((w * 8 + ks) * kUnit), 0));
    // pieces w + 4 i, i < PRE_SPLIT, of both tiles: LDS bytes < 4 PRE_SPLIT KiB, i.e. rows < 64 + halo
    constexpr int PRE_SPLIT = (64 * XPITCH + 1023) / 1024 / 4 + 1;
    static_assert(4 * PRE_SPLIT * 1024 >= 64 * XPITCH && PRE_SPLIT <= XP_PER_WAVE, "row pass 0 pieces");
    tile_dma_range(p.att, p.att_bytes, p.as, ATT_OFF, 0, PRE_SPLIT);
    tile_dma_range(a.x, a.x_bytes, a.xs, X_OFF, 0, PRE_SPLIT);
    tile_dma_range(p.att, p.att_bytes, p.as, ATT_OFF, PRE_SPLIT, XP_PER_WAVE);
    tile_dma_range(a.x, a.x_bytes, a.xs, X_OFF, PRE_SPLIT, XP_PER_WAVE);
    stamp(21);
    // everything but the second-half pieces (2 (XP_PER_WAVE - PRE_SPLIT) per wave, the youngest)
    __builtin_amdgcn_s_waitcnt(vm_imm(2 * (XP_PER_WAVE - PRE_SPLIT)));
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
    stamp(22);
    float *red0 = reinterpret_cast<float *>(smem + RED0_OFF);
    static_for<(XROWS + 63) / 64>([&](auto PS) {
      constexpr int ps = decltype(PS)::value;
      if constexpr (ps == 1) {  // the second half of both tiles
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      f32x4 a0[4][4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) a0[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        bf16x8 fb[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const int r = min(64 * ps + 16 * mb + hr, XROWS - 1);  // rows past the tile: never stored
          fb[mb] = *reinterpret_cast<const bf16x8 *>(smem + ATT_OFF + r * XPITCH + ks * 64 + hq * 16);
        }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
          for (int jb = 0; jb < 4; ++jb)
            a0[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][jb], fb[mb], a0[jb][mb], 0, 0, 0);
      }
      // + bfc + residual; row statistics over the 4 waves' 64 columns each (jb outer: each LDS
      // vector read once per pass; per row the same summation order as row-major)
      float part[4] = {0.f, 0.f, 0.f, 0.f}, mean[4], var[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int n = w * 64 + jb * 16 + 4 * hq;
        const float4 bb = *reinterpret_cast<const float4 *>(smem + VEC0_OFF + 4 * n);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const int r = 64 * ps + 16 * mb + hr, gm = m0 - pad + r;
          const bool ok = r < XROWS && gm >= 0 && gm < M;
          bf16x4 xv = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
          if (ok) xv = *reinterpret_cast<const bf16x4 *>(smem + X_OFF + r * XPITCH + n * 2);
          f32x4 v = a0[jb][mb];
          v[0] = v[0] + bb.x + (float)xv[0];
          v[1] = v[1] + bb.y + (float)xv[1];
          v[2] = v[2] + bb.z + (float)xv[2];
          v[3] = v[3] + bb.w + (float)xv[3];
          a0[jb][mb] = v;
          part[mb] += (v[0] + v[1]) + (v[2] + v[3]);
        }
      }
      auto reduce4 = [&](float (&pv)[4], float (&tot)[4]) {
        float t[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) t[mb] = __shfl_xor(pv[mb], 16, 64);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) pv[mb] += t[mb];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) t[mb] = __shfl_xor(pv[mb], 32, 64);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) red0[(mb * 16 + hr) * 4 + w] = pv[mb] + t[mb];
        __builtin_amdgcn_s_waitcnt(kLgkm0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const float4 r4 = *reinterpret_cast<const float4 *>(red0 + (mb * 16 + hr) * 4);
          tot[mb] = (r4.x + r4.y) + (r4.z + r4.w);
        }
        __builtin_amdgcn_s_waitcnt(kLgkm0);
        __builtin_amdgcn_s_barrier();
      };
      reduce4(part, mean);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        mean[mb] *= 1.0f / kD;
        float ss = 0.f;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          f32x4 d = a0[jb][mb];
          d[0] -= mean[mb];
          d[1] -= mean[mb];
          d[2] -= mean[mb];
          d[3] -= mean[mb];
          a0[jb][mb] = d;
          ss += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
        }
        part[mb] = ss;
      }
      reduce4(part, var);
      float rstd[4], keep[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) rstd[mb] = 1.0f / sqrtf(var[mb] * (1.0f / kD) + p.eps1);
      // padded rows (t >= lens[b], the encoder's [B, L] form): h = masked_fill(LN1(.), 0)
      // (transformer/Layers.py:25-26), the zeros the FFN's conv taps read past a sequence's end
      if (a.lens != nullptr) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const int gm = m0 - pad + 64 * ps + 16 * mb + hr;
          if (gm >= 0 && gm < M) {
            const int bb = gm / T;
            keep[mb] = (int64_t)(gm - bb * T) < a.lens[bb] ? 1.0f : 0.0f;
          }
        }
      }
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int n = w * 64 + jb * 16 + 4 * hq;
        const float4 g = *reinterpret_cast<const float4 *>(smem + VEC0_OFF + 4 * (kD + n));
        const float4 be = *reinterpret_cast<const float4 *>(smem + VEC0_OFF + 4 * (2 * kD + n));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const int r = 64 * ps + 16 * mb + hr;
          const f32x4 d = a0[jb][mb];
          bf16x4 o;
          o[0] = (bf16)((d[0] * rstd[mb] * g.x + be.x) * keep[mb]);
          o[1] = (bf16)((d[1] * rstd[mb] * g.y + be.y) * keep[mb]);
          o[2] = (bf16)((d[2] * rstd[mb] * g.z + be.z) * keep[mb]);
          o[3] = (bf16)((d[3] * rstd[mb] * g.w + be.w) * keep[mb]);
          if (r < XROWS) *reinterpret_cast<bf16x4 *>(smem + X_OFF + r * XPITCH + n * 2) = o;
        }
      }
      stamp(23 + ps);
    });
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();  // every wave past its att reads: the vectors overwrite the region
    load_vectors();
    ring_start();
  }


  // ---- B fragments
  const int hrow0 = lane & 15;  // activation row (tile-relative) of block 0
  const int hi = lane >> 4;
  bf16x8 f0[MB], f1[MB];
  // GEMM1 fragment addresses of a tap: row (lane row + tap + 16 mb) of the x tile, channel group
  // hi; a masked row's address is 0 (the zero region). Computed once per tap; a unit (tap, ks)
  // reads base + 64 ks (an immediate offset).
  auto bases_x = [&](int tap, int (&ad)[MB]) {
    const int base = X_OFF + (hrow0 + tap) * XPITCH + hi * 16;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int keep = (FFN_ABLATE & 16) ? -1 : __builtin_amdgcn_sbfe(vmask[mb], tap, 1);
      ad[mb] = (base + mb * 16 * XPITCH) & keep;
    }
  };
  auto issue_x = [&](const int (&ad)[MB], auto KSI, bf16x8 (&f)[MB]) {
    if (FFN_ABLATE & 4) return;
    constexpr int off = decltype(KSI)::value * 64;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) f[mb] = *reinterpret_cast<const bf16x8 *>(smem + ad[mb] + off);
  };
  // GEMM2 unit q (32 hidden columns of the chunk)
  auto read_h = [&](int q, bf16x8 (&f)[MB]) {
    if (FFN_ABLATE & 4) return;
    const char *hp = smem + H_OFF + hrow0 * 512 + (xchunk(hrow0, 4 * q + hi) << 4);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) f[mb] = *reinterpret_cast<const bf16x8 *>(hp + mb * 8192);
  };

  f32x4 acc1[4][MB], acc2[4][MB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  auto mma = [&](f32x4 (&acc)[4][MB], const bf16x8 (&fa)[4], const bf16x8 (&fb)[MB]) {
    if (FFN_ABLATE & 1) return;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[jb], fb[mb], acc[jb][mb], 0, 0, 0);
  };
  auto bar = []() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // trace builds: 32 stamp slots per workgroup -- past the split-K partials in the workspace for the
  // split form (probe-sized workspace), else output row a.M - 1 - block (the packed capacity tail)
  auto trace_dump = [&](int last) {
    if (FFN_TRACE) {
      uint64_t *o = S > 1 ? reinterpret_cast<uint64_t *>(static_cast<char *>(p.part) + p.part_bytes + 256u * blockIdx.x)
                          : reinterpret_cast<uint64_t *>(static_cast<char *>(a.out) + (size_t)(a.M - 1 - blockIdx.x) * a.os * 2);
      for (int i = 0; i < 25; ++i) o[i] = *reinterpret_cast<const uint64_t *>(smem + SMEM + 8 * i);
      o[28] = t_entry;
      o[29] = (uint64_t)split;
      o[30] = (uint64_t)last;
      o[31] = (uint64_t)25;
    }
  };
  stamp(0);

  // chunk c's hidden slice: H[m][j] = bf16(relu(acc1 + b1)); lane holds 4 consecutive j of row m
  auto write_h = [&](int c) {
    float z;  // an opaque 0: a constant zero here makes the register allocator rotate acc1
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int j = w * 64 + jb * 16 + 4 * hi;  // hidden column inside the chunk
      const float4 bb = *reinterpret_cast<const float4 *>(smem + B1_OFF + 4 * (c * kChunk + j));
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const f32x4 v = acc1[jb][mb];
        bf16x4 o;
        o[0] = (bf16)fmaxf(v[0] + bb.x, 0.f);
        o[1] = (bf16)fmaxf(v[1] + bb.y, 0.f);
        o[2] = (bf16)fmaxf(v[2] + bb.z, 0.f);
        o[3] = (bf16)fmaxf(v[3] + bb.w, 0.f);
        const int m = hrow0 + mb * 16;
        *reinterpret_cast<bf16x4 *>(smem + H_OFF + m * 512 + (xchunk(m, j >> 3) << 4) + (j & 7) * 2) = o;
        acc1[jb][mb] = f32x4{z, z, z, z};
      }
    }
  };

  // x tile landed (the DEPTH * 4 weight loads behind it may stay in flight), b1 stored; visible
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * DEPTH) : "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  bar();
  stamp(1);
  int bxc[MB], bxn[MB];  // fragment bases of the current and the next tap
  bases_x(0, bxc);
  issue_x(bxc, std::integral_constant<int, 0>{}, f0);

  // GEMM1, tap by tap: 8 units (k-steps of 32 channels) per tap, unit k = 8 tap + ks in ring slot
  // ks % DEPTH. A unit reads the next unit's B fragments (LDS latency hidden behind its 28 MFMAs;
  // after ks 7 with the next tap's bases), then refills its slot with the unit DEPTH ahead (GEMM1,
  // or for the last tap's second half GEMM2 unit ks - 4 of this wave's rotated order). Units
  // alternate f0 / f1 by parity. After the last tap the read is of "tap KS" (masked: zeros).
  static_assert(DEPTH == 4 && kD / 32 == 8, "8 units per tap, 4-unit ring");
  auto unit1 = [&](auto KSI, int c, int tap) {
    constexpr int ks = decltype(KSI)::value, s = ks % DEPTH;
    if constexpr (ks + 1 < 8) {
      if constexpr (ks & 1)
        issue_x(bxc, std::integral_constant<int, ks + 1>{}, f0);
      else
        issue_x(bxc, std::integral_constant<int, ks + 1>{}, f1);
    } else {
      issue_x(bxn, std::integral_constant<int, 0>{}, f0);
    }
    if constexpr (ks & 1)
      mma(acc1, pa[s], f1);
    else
      mma(acc1, pa[s], f0);
    const uint32_t k1 = (uint32_t)(tap * 8 + ks + DEPTH) * (uint32_t)kUnit;
    if constexpr (ks + DEPTH < 8) {
      load_at(std::integral_constant<int, s>{}, base1(c) + k1);
    } else {
      const bool more = tap + 1 < KS;  // scalar select: GEMM1 of the next tap, or GEMM2
      load_at(std::integral_constant<int, s>{},
              more ? base1(c) + k1 : base2(c) + (uint32_t)(((2 * w + ks - DEPTH) & (NK2 - 1)) * kUnit));
    }
  };
#pragma nounroll
  for (int c = c0; c < cend; ++c) {
#pragma nounroll
    for (int tap = 0; tap < KS; ++tap) {
      bases_x(tap + 1, bxn);
      static_for<8>([&](auto KSI) { unit1(KSI, c, tap); });
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) bxc[mb] = bxn[mb];
    }
    // every wave is past its GEMM2 reads of the previous chunk's H: overwrite it. GEMM2 walks the
    // chunk's hidden columns starting at this wave's own block (units 2w, 2w + 1: its own writes,
    // no barrier); the barrier that makes the other waves' blocks visible comes after that first
    // unit, so it absorbs the skew between the waves' write_h instead of stalling on it.
    stamp(2 + 2 * (c - c0));
    bar();
    write_h(c);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    stamp(3 + 2 * (c - c0));
    read_h(2 * w, f0);
    const uint32_t next1 = c + 1 < cend ? base1(c + 1) : 0u;  // past the last unit: harmless reloads
    static_for<NK2>([&](auto Q) {
      constexpr int q = decltype(Q)::value;  // this wave's q-th GEMM2 unit: hidden columns 32 * qq
      constexpr int s = q % DEPTH;
      if constexpr (q == 1) {
        __builtin_amdgcn_s_waitcnt(kLgkm0);
        bar();  // every wave's H block written and visible
      }
      const int qn = (2 * w + q + 1) & (NK2 - 1);
      if constexpr (q + 1 == NK2) {  // the next chunk's first unit (x is never overwritten)
        bases_x(0, bxc);
        issue_x(bxc, std::integral_constant<int, 0>{}, f0);
      }
      else if constexpr (q & 1)
        read_h(qn, f0);
      else
        read_h(qn, f1);
      if constexpr (q & 1)
        mma(acc2, pa[s], f1);
      else
        mma(acc2, pa[s], f0);
      if constexpr (q + DEPTH < NK2)
        load_at(std::integral_constant<int, s>{}, base2(c) + (uint32_t)(((2 * w + q + DEPTH) & (NK2 - 1)) * kUnit));
      else
        load_at(std::integral_constant<int, s>{}, next1 + (uint32_t)((q + DEPTH - NK2) * kUnit));
    });
  }

  // ---- LN epilogue straight from the Y^T accumulators (Layers.py:28 residual + LayerNorm, the
  // padding mask, the speaker / emotion adds). Lane (wave w, lane l) holds rows mb*16 + (l & 15),
  // columns 64w + 16nb + 4(l >> 4) + i; a row's 256 values live in 4 lanes of each of the 4 waves:
  // partial sums over the lane's 16 values, a butterfly over l >> 4, then the 4 waves' partials
  // through LDS. The residual x rows are still in the LDS x tile; the bf16 result is staged in
  // the H region and written out as whole 512-byte rows.
  stamp(2 + 2 * NCH);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the harmless past-the-end weight loads
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  stamp(4 + 2 * NCH);
  if (S > 1) {
    // split-hidden hand-off (as conv_gemm.hip's splitk_fixup): every split stores its partial Y^T
    // with sc1 (write-through) 16-byte stores, drains, and one lane adds to the tile's counter; the
    // split whose add comes last resets the counter, acquires, and sums the partials in split order
    // (its own from registers). The other splits are done.
    const rsrc_t pr = make_rsrc(p.part, p.part_bytes);
    auto pofs = [&](int sp, int nb, int mb) {
      return (uint32_t)(tile * S + sp) * (uint32_t)kPartBytes + (uint32_t)((((w * 4 + nb) * MB + mb) * 64 + lane) * 16);
    };
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, acc2[nb][mb]),
                                               pr, pofs(split, nb, mb), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *flag = reinterpret_cast<int *>(smem + RED_OFF);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) {
        __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for the next launch
        // no acquire (an L1 invalidate, ~1.7 us): every byte handed off is stored AND loaded with
        // 16-byte sc1 buffer ops (L1 bypassed both ways), each storing wave drained vmcnt before the
        // barrier behind which one lane adds, the last adder is told by its add's return value and
        // the other waves load behind the barrier it joins, one workgroup per CU -- the measured
        // sc1 hand-off of MI355X_MICROARCH.md (inter-workgroup visibility, first row).
        // FS2_FFN_ACQUIRE=1 restores the fence (A/B).
        if (p.acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      *flag = last;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(19);
    if (FFN_TRACE && !*flag) {  // trace builds: the stamps of a split that hands off and exits
      if (tid == 0) trace_dump(0);
    }
    if (!*flag) return;
    __syncthreads();  // flag read by every wave before the epilogue reuses the slot
    // sum in split order into the dead H^T accumulators. MB = 4: every other split's partial is
    // loaded at once (3 x 16 x 4 registers), one memory round trip; MB = 7: one other split's 28
    // loads in flight at a time (a per-load branch on the split index serialised every load's
    // full latency)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc1[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (MB <= 4) {
      f32x4 v[3][4][MB];
      static_for<3>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if (j < S - 1) {
          const int sp = j + (j >= split ? 1 : 0);
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              v[j][nb][mb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, pofs(sp, nb, mb), 0, 16));
        }
      });
      static_for<4>([&](auto SP) {
        constexpr int sp = decltype(SP)::value;
        constexpr int jlo = sp < 3 ? sp : 2, jhi = sp > 0 ? sp - 1 : 0;
        if (sp < S) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              acc1[nb][mb] += sp < split ? v[jlo][nb][mb] : (sp == split ? acc2[nb][mb] : v[jhi][nb][mb]);
        }
      });
    } else {
      for (int sp = 0; sp < S; ++sp) {
        if (sp == split) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc1[nb][mb] += acc2[nb][mb];
        } else {
          f32x4 v[4][MB];
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              v[nb][mb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, pofs(sp, nb, mb), 0, 16));
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc1[nb][mb] += v[nb][mb];
        }
      }
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc2[nb][mb] = acc1[nb][mb];
    stamp(20);
  }
  {
    float *red = reinterpret_cast<float *>(smem + RED_OFF);
    const float inv_n = 1.0f / 256.0f;
    float4 b2v[4], gv[4], bev[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = w * 64 + nb * 16 + 4 * hi;
      b2v[nb] = *reinterpret_cast<const float4 *>(smem + EP_OFF + 4 * n);
      gv[nb] = *reinterpret_cast<const float4 *>(smem + EP_OFF + 4 * (kD + n));
      bev[nb] = *reinterpret_cast<const float4 *>(smem + EP_OFF + 4 * (2 * kD + n));
    }
    // v = acc + b2 + x (into acc2), row partial sums
    float part[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int xr = mb * 16 + hrow0 + pad;  // the row's own x in the tile
      float sum = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int n = w * 64 + nb * 16 + 4 * hi;
        const bf16x4 xv = *reinterpret_cast<const bf16x4 *>(smem + X_OFF + xr * XPITCH + n * 2);
        f32x4 v = acc2[nb][mb];
        v[0] = v[0] + b2v[nb].x + (float)xv[0];
        v[1] = v[1] + b2v[nb].y + (float)xv[1];
        v[2] = v[2] + b2v[nb].z + (float)xv[2];
        v[3] = v[3] + b2v[nb].w + (float)xv[3];
        acc2[nb][mb] = v;
        sum += (v[0] + v[1]) + (v[2] + v[3]);
      }
      part[mb] = sum;
    }
    // row statistic: 4 lanes (l >> 4) per wave, then the 4 waves through LDS
    auto row_reduce = [&](float (&pv)[MB], float (&tot)[MB]) {
      // all rows' shuffles issued together (one LDS round trip per level, not one per row); the
      // 4 lanes of a row store the same sum to the same slot (no divergent branch)
      float t[MB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) t[mb] = __shfl_xor(pv[mb], 16, 64);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) pv[mb] += t[mb];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) t[mb] = __shfl_xor(pv[mb], 32, 64);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) red[(mb * 16 + hrow0) * 4 + w] = pv[mb] + t[mb];
      __syncthreads();
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const float4 r = *reinterpret_cast<const float4 *>(red + (mb * 16 + hrow0) * 4);
        tot[mb] = (r.x + r.y) + (r.z + r.w);
      }
      __syncthreads();  // red is reused by the next statistic
    };
    float mean[MB], var[MB];
    stamp(14);
    row_reduce(part, mean);
    stamp(15);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      mean[mb] *= inv_n;
      float ss = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        f32x4 d = acc2[nb][mb];
        d[0] -= mean[mb];
        d[1] -= mean[mb];
        d[2] -= mean[mb];
        d[3] -= mean[mb];
        acc2[nb][mb] = d;
        ss += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
      }
      part[mb] = ss;
    }
    stamp(16);
    row_reduce(part, var);
    stamp(17);
    // y = d * rstd * gamma + beta; padded rows: mask, then + addvec (FastSpeech2.forward adds the
    // speaker / emotion vectors to every frame); bf16 into the H region (free since GEMM2 ended).
    // The padded-row extras are a separate instantiation: per-element branches for them made the
    // packed (decoder) path's epilogue several times longer.
    auto finish = [&](auto PADDED) {
      constexpr bool padded = decltype(PADDED)::value;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const float rstd = 1.0f / sqrtf(var[mb] * inv_n + a.eps);
        const int m = mb * 16 + hrow0;
        bool masked = false;
        int bb = 0;
        if constexpr (padded) {
          bb = (m0 + m) / T;
          masked = (padmask >> mb) & 1;
        }
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int n = w * 64 + nb * 16 + 4 * hi;
          const f32x4 d = acc2[nb][mb];
          float y[4] = {d[0] * rstd * gv[nb].x + bev[nb].x, d[1] * rstd * gv[nb].y + bev[nb].y,
                        d[2] * rstd * gv[nb].z + bev[nb].z, d[3] * rstd * gv[nb].w + bev[nb].w};
          if constexpr (padded) {
            if (masked) y[0] = y[1] = y[2] = y[3] = 0.f;
            if (a.av1 != nullptr) {
              const float4 v1 = *reinterpret_cast<const float4 *>(a.av1 + (int64_t)bb * kD + n);
              y[0] += v1.x; y[1] += v1.y; y[2] += v1.z; y[3] += v1.w;
            }
            if (a.av2 != nullptr) {
              const float4 v2 = *reinterpret_cast<const float4 *>(a.av2 + (int64_t)bb * kD + n);
              y[0] += v2.x; y[1] += v2.y; y[2] += v2.z; y[3] += v2.w;
            }
          }
          bf16x4 o;
          o[0] = (bf16)y[0];
          o[1] = (bf16)y[1];
          o[2] = (bf16)y[2];
          o[3] = (bf16)y[3];
          *reinterpret_cast<bf16x4 *>(smem + H_OFF + m * 512 + (xchunk(m, n >> 3) << 4) + (n & 7) * 2) = o;
        }
      }
    };
    if (a.lens != nullptr || a.av1 != nullptr || a.av2 != nullptr)
      finish(std::true_type{});
    else
      finish(std::false_type{});
    __syncthreads();
    stamp(18);
    // whole rows out: 16-byte chunks, 32 per row
    const uint32_t orow = (uint32_t)a.os * 2u;
    char *ob = static_cast<char *>(a.out);
#pragma unroll 2
    for (int i = tid; i < BM * 32; i += 256) {
      const int m = i >> 5, ch = i & 31;
      if (m0 + m < M) {
        const uint4 v = *reinterpret_cast<const uint4 *>(smem + H_OFF + m * 512 + (xchunk(m, ch) << 4));
        if (p.out_sc1)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                 make_rsrc(ob, 0x7fffffffu), (uint32_t)((m0 + m) * orow + ch * 16), 0, 16);
        else
          *reinterpret_cast<uint4 *>(ob + (size_t)(m0 + m) * orow + ch * 16) = v;
      }
    }
    // ---- the next block's Q|K|V projection (transformer/SubLayers.py:39-41 of block i+1) while
    // y is still on chip: GEMM3 Q|K|V^T[n, m] = sum_c Wq[n, c] . y[m, c] in passes of 256 output
    // columns (wave w: 64 of them, the accumulators of the dead H^T registers), y read from the H
    // region exactly as GEMM2 read H, weights through the same register ring; + bias, bf16,
    // staged in the x region (pitch 528: the 8-byte column writes of 16 rows conflict-free) and
    // stored as whole 512-byte row segments. Saves the Q|K|V launch's re-read of y and its tiles.
    if (p.wq != nullptr) {
      const rsrc_t qr = make_rsrc(p.wq, p.wq_bytes);
      auto qload = [&](auto S, uint32_t so) {
        constexpr int s = decltype(S)::value;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          auto v = __builtin_amdgcn_raw_buffer_load_b128(qr, lane_off + jb * 1024, so, 0);
          pa[s][jb] = __builtin_bit_cast(bf16x8, v);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      constexpr int SPITCH = 528;
      const uint32_t qrow = (uint32_t)p.qs * 2u;
      char *qb = reinterpret_cast<char *>(p.qkv);
      const int npass = p.nq / 256;
      auto qbase = [&](int ps) { return (uint32_t)((ps * 4 + w) * 8) * (uint32_t)kUnit; };
      // raw barrier: LDS traffic retired, global stores left in flight (they overlap the next pass)
      auto lbar = [&]() {
        __builtin_amdgcn_s_waitcnt(kLgkm0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<DEPTH>([&](auto I) { qload(I, qbase(0) + (uint32_t)(decltype(I)::value * kUnit)); });
#pragma nounroll
      for (int ps = 0; ps < npass; ++ps) {
        const uint32_t base = qbase(ps);
        float z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) acc1[jb][mb] = f32x4{z, z, z, z};
        read_h(0, f0);
        static_for<8>([&](auto Q) {
          constexpr int q = decltype(Q)::value, sl = q % DEPTH;
          if constexpr (q + 1 < 8) {
            if constexpr (q & 1)
              read_h(q + 1, f0);
            else
              read_h(q + 1, f1);
          }
          if constexpr (q & 1)
            mma(acc1, pa[sl], f1);
          else
            mma(acc1, pa[sl], f0);
          if constexpr (q + DEPTH < 8)
            qload(std::integral_constant<int, sl>{}, base + (uint32_t)((q + DEPTH) * kUnit));
          else  // the next pass's first units (past the last pass: harmless reloads of pass 0)
            qload(std::integral_constant<int, sl>{},
                  (ps + 1 < npass ? qbase(ps + 1) : qbase(0)) + (uint32_t)((q + DEPTH - 8) * kUnit));
        });
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          const int c = w * 64 + jb * 16 + 4 * hi;  // column inside this pass
          const float4 bb = *reinterpret_cast<const float4 *>(p.bq + ps * 256 + c);
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            const f32x4 v = acc1[jb][mb];
            bf16x4 o;
            o[0] = (bf16)(v[0] + bb.x);
            o[1] = (bf16)(v[1] + bb.y);
            o[2] = (bf16)(v[2] + bb.z);
            o[3] = (bf16)(v[3] + bb.w);
            *reinterpret_cast<bf16x4 *>(smem + X_OFF + (hrow0 + mb * 16) * SPITCH + c * 2) = o;
          }
        }
        lbar();
#pragma unroll 2
        for (int i = tid; i < BM * 32; i += 256) {
          const int m = i >> 5, ch = i & 31;
          if (m0 + m < M) {
            const uint4 v = *reinterpret_cast<const uint4 *>(smem + X_OFF + m * SPITCH + ch * 16);
            if (p.out_sc1)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                     make_rsrc(qb, 0x7fffffffu),
                                                     (uint32_t)((m0 + m) * qrow + ps * 512 + ch * 16), 0, 16);
            else
              *reinterpret_cast<uint4 *>(qb + (size_t)(m0 + m) * qrow + ps * 512 + ch * 16) = v;
          }
        }
        lbar();  // the staging region is rewritten by the next pass
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the harmless past-the-end reloads
    }
  }
  stamp(5 + 2 * NCH);
  if (FFN_TRACE) {
    stamp(3 + 2 * NCH);
    __syncthreads();
    if (tid == 0) trace_dump(1);
  }
}

}  // namespace

extern "C" int fs2_ffn(const fs2_ffn_desc *d, fs2_stream_t stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->b1 == nullptr || d->b2 == nullptr ||
      d->ln_gamma == nullptr || d->ln_beta == nullptr || d->out == nullptr)
    return FS2_EINVAL;
  if (d->B < 0 || d->T < 0 || d->x_row_stride < kD || (d->x_row_stride & 7) || d->out_row_stride < kD ||
      (d->out_row_stride & 7))
    return FS2_EINVAL;
  if (d->D != kD || !(d->F == 1024 || d->F == 512) || !(d->KS == 9 || d->KS == 3) || d->pad < 0 ||
      d->pad > d->KS - 1)
    return FS2_EUNSUPPORTED;
  if ((d->rows_dev == nullptr) != (d->row_pos == nullptr)) return FS2_EINVAL;
  if (d->rows_dev != nullptr && (d->lens != nullptr || d->addvec1 != nullptr || d->addvec2 != nullptr))
    return FS2_EINVAL;
  if (d->x == d->out) return FS2_EINVAL;  // other tiles re-read x rows (halo, residual)
  const int S = d->nsplit <= 1 ? 1 : d->nsplit;
  if (!(S == 1 || S == 2 || S == 4) || S > d->F / kChunk) return FS2_EINVAL;
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 > 0x7fffff00LL) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;
  const int64_t xb = M64 * d->x_row_stride * 2;
  const int64_t wb = ffn_weight_elems(d->KS, d->F) * 2;
  if (xb >= (1LL << 31)) return FS2_EUNSUPPORTED;

  FfnArgs p{};
  ConvArgs &a = p.e;
  a = ConvArgs{};
  a.x = d->x;
  a.xs = d->x_row_stride;
  a.w = d->w;
  a.bias = d->b2;
  a.B = d->B;
  a.T = d->T;
  a.Cin = kD;
  a.Cin_pad = kD;
  a.N = kD;
  a.KS = d->KS;
  a.pad = d->pad;
  a.M = (int)M64;
  a.epi = FS2_EPI_RES_LN;
  a.res = d->x;
  a.res_dt = FS2_BF16;
  a.rs = d->x_row_stride;
  a.gamma = d->ln_gamma;
  a.beta = d->ln_beta;
  a.eps = d->ln_eps;
  a.lens = d->lens;
  a.av1 = d->addvec1;
  a.av2 = d->addvec2;
  a.out = d->out;
  a.out_dt = FS2_BF16;
  a.os = d->out_row_stride;
  a.rows_dev = d->rows_dev;
  a.row_pos = reinterpret_cast<const int2 *>(d->row_pos);
  a.out_scale = 1.0f;
  a.ln_pairs = 1;
#ifdef FFN_EPI_DBG
  a.dbg = FFN_EPI_DBG;  // analysis builds: conv_common.h epilogue ablation bits
#endif
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.b1 = d->b1;
  p.w_bytes = (uint32_t)wb;
  if (d->wqkv != nullptr) {
    if (d->bqkv == nullptr || d->qkv_out == nullptr || d->nqkv <= 0 || (d->nqkv % 256) ||
        d->qkv_row_stride < d->nqkv || (d->qkv_row_stride & 7) || d->qkv_out == d->x || d->qkv_out == d->out)
      return FS2_EINVAL;
    p.wq = reinterpret_cast<const bf16 *>(d->wqkv);
    p.bq = d->bqkv;
    p.qkv = reinterpret_cast<bf16 *>(d->qkv_out);
    p.qs = d->qkv_row_stride;
    p.nq = d->nqkv;
    p.wq_bytes = (uint32_t)((int64_t)d->nqkv * kD * 2);
  }
  const bool pre = d->pre_att != nullptr;
  if (pre) {
    if (d->pre_w == nullptr || d->pre_b == nullptr || d->pre_gamma == nullptr || d->pre_beta == nullptr ||
        d->pre_att_row_stride < kD || (d->pre_att_row_stride & 7) || d->pre_att == d->out)
      return FS2_EINVAL;
    // packed launches (the decoder: unsplit 112- or 64-row tiles, or 96-row tiles x 2 splits when
    // free-running -- every split of a tile computes the prologue) or padded [B, T] rows with
    // lengths, 64-row tiles in the split-hidden form (the encoder)
    const bool dec_form = d->rows_dev != nullptr;
    const bool enc_form = d->rows_dev == nullptr && d->tile_rows == 64;
    if (!(dec_form || enc_form) || d->KS != 9 || d->F != 1024) return FS2_EUNSUPPORTED;
    const int64_t ab = M64 * d->pre_att_row_stride * 2;
    if (ab >= (1LL << 31)) return FS2_EUNSUPPORTED;
    p.att = reinterpret_cast<const bf16 *>(d->pre_att);
    p.as = d->pre_att_row_stride;
    p.att_bytes = (uint32_t)ab;
    p.wfc = reinterpret_cast<const bf16 *>(d->pre_w);
    p.bfc = d->pre_b;
    p.g1 = d->pre_gamma;
    p.be1 = d->pre_beta;
    p.eps1 = d->pre_eps;
  }
  if (d->rows_max < 0 || !(d->tile_rows == 0 || d->tile_rows == 112 || d->tile_rows == 96 || d->tile_rows == 64))
    return FS2_EINVAL;
  const int MB = d->tile_rows == 64 ? 4 : d->tile_rows == 96 ? 6 : 7, BM = 16 * MB;
  if (MB == 6 && (d->KS != 9 || d->F != 1024)) return FS2_EUNSUPPORTED;  // instantiated for the model's FFN only
  const int64_t kPartBytes = part_bytes(MB);
  const int64_t Mg = (d->rows_dev != nullptr && d->rows_max > 0 && d->rows_max < M64) ? d->rows_max : M64;
  a.M = (int)Mg;
  const int ntiles = (int)((Mg + BM - 1) / BM);
  int nwg = ntiles;
  p.nsplit = S;
  p.ntiles = ntiles;
  static const int acquire = [] {
    const char *e = getenv("FS2_FFN_ACQUIRE");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  p.acquire = acquire;
  static const int out_sc1 = [] {
    const char *e = getenv("FS2_OUT_SC1");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  p.out_sc1 = out_sc1;
  static const int ffn_prefetch = [] {
    const char *e = getenv("FS2_FFN_PREFETCH");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  p.prefetch = ffn_prefetch;
  if (S > 1) {
    if (d->splitk_ws == nullptr || ntiles > 1024 ||
        d->splitk_ws_bytes < 4096 + (int64_t)ntiles * S * kPartBytes + (FFN_TRACE ? 256LL * (ntiles * S + 8) : 0) ||
        (int64_t)ntiles * S * kPartBytes >= (1LL << 31))
      return FS2_EINVAL;
    p.cnt = static_cast<int *>(d->splitk_ws);
    p.part = static_cast<char *>(d->splitk_ws) + 4096;
    p.part_bytes = (uint32_t)((int64_t)ntiles * S * kPartBytes);
    nwg = (ntiles * S + 7) & ~7;
  }
  const int nch = d->F / kChunk;
  hipStream_t s = as_stream(stream);
  // instantiated shapes: kernel 9 (model.yaml conv_kernel_size [9, 1]) or 3, F = 1024 or 512
  auto go = [&](auto KSC, auto NCHC) {
    constexpr int ks = decltype(KSC)::value, nc = decltype(NCHC)::value;
    if (MB == 4)
      hipLaunchKernelGGL((ffn_fused_kernel<ks, nc, 4>), dim3(nwg), dim3(256), 0, s, p);
    else if constexpr (ks == 9 && nc == 4) {
      if (MB == 6)
        hipLaunchKernelGGL((ffn_fused_kernel<9, 4, 6>), dim3(nwg), dim3(256), 0, s, p);
      else
        hipLaunchKernelGGL((ffn_fused_kernel<ks, nc, 7>), dim3(nwg), dim3(256), 0, s, p);
    } else
      hipLaunchKernelGGL((ffn_fused_kernel<ks, nc, 7>), dim3(nwg), dim3(256), 0, s, p);
  };
  using I9 = std::integral_constant<int, 9>;
  using I3 = std::integral_constant<int, 3>;
  using C4 = std::integral_constant<int, 4>;
  using C2 = std::integral_constant<int, 2>;
  if (pre && MB == 4)
    hipLaunchKernelGGL((ffn_fused_kernel<9, 4, 4, true>), dim3(nwg), dim3(256), 0, s, p);
  else if (pre && MB == 6)
    hipLaunchKernelGGL((ffn_fused_kernel<9, 4, 6, true>), dim3(nwg), dim3(256), 0, s, p);
  else if (pre)
    hipLaunchKernelGGL((ffn_fused_kernel<9, 4, 7, true>), dim3(nwg), dim3(256), 0, s, p);
  else if (d->KS == 9 && nch == 4)
    go(I9{}, C4{});
  else if (d->KS == 9 && nch == 2)
    go(I9{}, C2{});
  else if (d->KS == 3 && nch == 4)
    go(I3{}, C4{});
  else if (d->KS == 3 && nch == 2)
    go(I3{}, C2{});
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int64_t fs2_ffn_weight_elems(int KS, int F) { return ffn_weight_elems(KS, F); }
