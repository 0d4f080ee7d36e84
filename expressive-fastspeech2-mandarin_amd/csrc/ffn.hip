// PositionwiseFeedForward + residual + LayerNorm + padding mask as ONE kernel (gfx950 / CDNA4):
//
//   f = relu(Conv1d_k9(x; w1) + b1)              [rows, 1024]   -- never leaves the CU
//   y = LN(f . w2^T + b2 + x) ; masked ; (+ addvec)               -- transformer/SubLayers.py:85-93
//
// Why one kernel: as two launches the 1024-wide hidden f is written to HBM by the k=9 conv and
// read back by the k=1 conv (cfg2 decoder: 51 MB each way per block), and the k=1 conv + LN runs
// as its own latency-bound launch (18 % of MFMA peak). Here a workgroup owns BM = 112 rows for
// the whole FFN and walks the hidden dimension in 4 chunks of 256 columns:
//
//   for chunk c:  GEMM1  H^T[j, m] = sum_{cb, tap} W1[c*256 + j, tap, cb*64 ...] . X[m + tap - pad, ...]
//                 H = relu(H^T + b1) -> bf16 -> LDS [112 x 256]            (chunk of f, on chip)
//                 GEMM2  Y^T[n, m] += sum_j W2[n, c*256 + j] . H[m, j]      (accumulated in registers)
//   LN epilogue on Y (through LDS, conv_common.h's epilogue).
//
// Both GEMMs put the WEIGHTS on the MFMA A side (rows j / n, 16 per block) and the activations on
// the B side (columns m). 4 waves, one per SIMD, 512 registers each: wave w owns weight rows
// 64w .. 64w+63 of every k-step and all 112 activation rows, so its two accumulators (H^T and
// Y^T, 4 x 7 blocks of 16x16 f32 each) sit in the accumulator registers for the whole kernel.
//
// Pipeline (a "unit" = one 32-channel k-step: 28 MFMAs per wave). Each wave streams ITS OWN
// weight rows through its own 6-unit LDS-DMA ring (4 KiB per unit, the unit 5 ahead in flight) and
// reads the next unit's fragments while the current unit's MFMAs run (two fragment register
// sets), so the weight stream needs no workgroup barrier at all: the waves run free. Barriers
// only where data is shared: the x rows of a 64-channel block (the tile + the taps' halo, 120 x
// 128 B, DMA'd by all four waves once per (chunk, block) and read shifted by the tap) and the
// hidden slice H. A fragment whose shifted row leaves its sequence reads a zero slot instead.
// LDS: rings 96 KiB + H 56 KiB (4 column blocks of 64) + b1 4 KiB; the two halo buffers live
// inside the H region, which is free while GEMM1 runs (the next chunk's first halo goes into H's
// column blocks 0-1 once GEMM2 has read them). One workgroup per CU; the LN epilogue reuses it.
#include <type_traits>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

#ifndef FFN_ABLATE
#define FFN_ABLATE 0  // analysis builds only: bit 0 no MFMAs, bit 1 no weight DMA, bit 2 no fragment reads
#endif

constexpr int kD = 256;            // d_model (encoder_hidden / decoder_hidden)
constexpr int kChunk = 256;        // hidden columns per chunk
constexpr int kNU = 6;             // units in each wave's weight ring
constexpr int kUnitW = 64 * 64;    // one wave's unit: 64 weight rows x 32 bf16 channels (4 KiB)

struct FfnArgs {
  ConvArgs e;          // x / rows / LN epilogue fields (conv_common.h); e.w unused
  const bf16 *w;       // fs2_ffn_desc.w: F rows of W1 ([KS][256]) then 256 rows of W2 ([F]), pitch ffn_pitch
  const float *b1;     // [F]
  uint32_t w_bytes;
};

// row pitch (elements) of the packed FFN weights: one pitch for both matrices, so a weight row of
// either GEMM is the same lane offset (only the scalar unit offset differs)
constexpr int ffn_pitch(int KS, int F) { return KS * 256 > F ? KS * 256 : F; }

// physical 16-byte chunk of logical chunk c (0..3) in a 64-byte ring row r: rows r and r + 8 swap
// chunk pairs, which makes the 16-row fragment reads (ds_read_b128 lane groups) conflict-free
__device__ __forceinline__ int ring_chunk(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

template <int MB>
struct FragsT {
  bf16x8 a[4];   // weight rows: 4 blocks of 16
  bf16x8 b[MB];  // activation rows: MB blocks of 16
};

// lgkmcnt(0) as a real s_waitcnt the compiler's wait-count pass sees (an asm one is opaque to it,
// so it would keep counting the previous unit's fragment reads as outstanding): gfx9 simm16 =
// vmcnt 63 (bits 3:0 and 15:14), expcnt 7, lgkmcnt 0
constexpr int kLgkm0 = 0xC07F;

template <int HB, int KS, int NCH>
__global__ __launch_bounds__(256, 1) void ffn_fused_kernel(FfnArgs p) {
  constexpr int BM = 16 * HB, MB = HB;
  static_assert(HB <= 7, "LDS sized for <= 112 rows");
  constexpr int HALO_BYTES = 16 * 1024;             // (BM + 8) x 128 B, 16 pieces: 4 per wave
  static_assert(BM + 8 <= 128, "halo pieces");
  constexpr int RING_OFF = 0;                       // wave w's ring at w * kNU * kUnitW
  constexpr int H_OFF = 4 * kNU * kUnitW;           // H: 4 column blocks of [BM rows][128 B]
  constexpr int H_BLK = BM * 128;
  constexpr int B1_OFF = H_OFF + 4 * H_BLK;
  constexpr int ZERO_OFF = B1_OFF + 4096;           // 16 zero bytes: masked halo fragments read here
  constexpr int EPI_LD = 256 + 4;
  constexpr int SMEM0 = ZERO_OFF + 16;
  constexpr int SMEM = SMEM0 > BM * EPI_LD * 4 ? SMEM0 : BM * EPI_LD * 4;
  static_assert(SMEM <= 163840, "LDS");
  static_assert(2 * HALO_BYTES <= 4 * H_BLK && HALO_BYTES <= 2 * H_BLK, "halo buffers inside H");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const ConvArgs &a = p.e;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // weight-row quarter (64 rows)
  const int M = a.rows_dev != nullptr ? *a.rows_dev : a.M;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int pad = a.pad, T = a.T;
  constexpr int F = NCH * kChunk;

  // ---- b1 -> LDS (plain loads before any LDS-DMA is in flight), the zero slot
  for (int i = tid; i < F / 4; i += 256)
    *reinterpret_cast<float4 *>(smem + B1_OFF + 16 * i) = reinterpret_cast<const float4 *>(p.b1)[i];
  if (tid == 0) *reinterpret_cast<float4 *>(smem + ZERO_OFF) = make_float4(0.f, 0.f, 0.f, 0.f);

  // ---- tap validity of this lane's activation rows (sequence position / length)
  int tpos[MB], tlen[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + mb * 16 + (lane & 15);
    if (m >= M) {
      tpos[mb] = 0;
      tlen[mb] = 0;  // never valid (rows past M are not stored)
    } else if (a.row_pos != nullptr) {
      const int2 q = a.row_pos[m];
      tpos[mb] = q.x;
      tlen[mb] = q.y;
    } else {
      tpos[mb] = m % T;
      tlen[mb] = T;
    }
  }
  int tw = 0, lw = 0;
  if (a.row_pos != nullptr) {
    const int2 q = a.row_pos[m0];
    tw = q.x;
    lw = q.y;
  } else {
    tw = m0 % T;
    lw = T;
  }
  const bool tile_inside = tw + BM <= lw && m0 + BM <= M;
  // taps whose shifted rows may leave a sequence somewhere in the tile (bit tap): masked reads
  uint32_t need_mask = 0;
#pragma unroll
  for (int tap = 0; tap < KS; ++tap) {
    const int sh = tap - pad;
    if (!(tile_inside && tw + sh >= 0 && tw + BM - 1 + sh < lw)) need_mask |= 1u << tap;
  }
  // consume the row_pos loads here: a first use behind the LDS-DMA stream would drain it
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) asm volatile("" ::"v"(tpos[mb]), "v"(tlen[mb]));

  // ---- DMA addressing
  constexpr int PITCH = ffn_pitch(KS, F);
  constexpr uint32_t wrow = (uint32_t)PITCH * 2u, w2off = (uint32_t)F * wrow;
  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t xrow = (uint32_t)a.xs * 2u;
  auto glds = [&](rsrc_t rs, char *dst, uint32_t off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)dst, 16, off, 0, 0, 0);
  };
  // Weight units: 1 KiB pieces of 16 rows x 64 B, lane-linear image; lane l -> row 16i + l/4 of
  // the wave's 64, physical chunk l & 3 (the ring_chunk swizzle applied on the source address)
  const int urow = lane >> 2;
  const uint32_t ulo = (uint32_t)(64 * w + urow) * wrow + (uint32_t)ring_chunk(urow, lane & 3) * 16u;
  // Unit schedule: units come in pairs = 64-channel k-steps (+64 B for the second half). Pairs of
  // a chunk: GEMM1 pr = cb * KS + tap (pr < NP1), then GEMM2 pr = NP1 + qp (64 hidden columns).
  // Lane pr of ptab_off / ptab_str holds pair pr's byte offset in chunk 0 and the chunk stride:
  // the producer reads both with v_readlane instead of decoding the unit.
  constexpr int NP1 = 4 * KS, NPC = NP1 + kChunk / 64;
  static_assert(NPC <= 64, "one table lane per pair");
  const int tl = lane < NPC ? lane : NPC - 1;
  const uint32_t ptab_off = tl < NP1 ? (uint32_t)((tl % KS) * (2 * kD) + (tl / KS) * 128)
                                     : w2off + (uint32_t)(128 * (tl - NP1));
  const uint32_t ptab_str = tl < NP1 ? (uint32_t)kChunk * wrow : (uint32_t)(2 * kChunk);
  char *const ring = smem + RING_OFF + w * (kNU * kUnitW);
  // unit `half` of pair (c, pr) into ring slot `slot` (4 pieces). Past the last unit (c == NCH) the
  // offsets run into W2 or past the buffer (zeros): harmless loads that keep every unit's vmcnt
  // count equal.
  auto issue_unit = [&](int c, int pr, int half, int slot) {
    if (FFN_ABLATE & 2) return;
    const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)ptab_off, pr) +
                         (uint32_t)c * (uint32_t)__builtin_amdgcn_readlane((int)ptab_str, pr) +
                         (uint32_t)(half * 64) + ulo;
    char *dst = ring + slot * kUnitW;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds(wr, dst + i * 1024, off + (uint32_t)(16 * i) * wrow);
  };
  // halo of channel block cb: rows m0 - pad .. m0 + BM + KS - 2, 128 B (64 channels) each, into
  // halo buffer `buf` (inside the H region); 4 pieces of 8 rows per wave
  const int prow = lane >> 3, plc = (lane & 7) ^ ((lane >> 3) & 7);
  auto issue_halo = [&](int cb, int buf) {
    char *dst = smem + H_OFF + buf * HALO_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = w + 4 * i;
      const int hr = 8 * pc + prow;
      const int gm = m0 - pad + hr;
      const bool ok = hr < BM + KS - 1 && gm >= 0 && gm < M;
      glds(xr, dst + pc * 1024, ok ? (uint32_t)gm * xrow + (uint32_t)(cb * 64 + plc * 8) * 2u : kOOB);
    }
  };

  // ---- fragment reads
  const int aoff = (lane & 15) * 64 + ring_chunk(lane & 15, lane >> 4) * 16;  // + 1 KiB per block
  const int hrow0 = lane & 15;  // activation row (tile-relative) of block 0
  auto read_a = [&](int slot, FragsT<MB> &f) {
    const char *st = ring + slot * kUnitW + aoff;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) f.a[jb] = *reinterpret_cast<const bf16x8 *>(st + jb * 1024);
  };
  // GEMM1 unit (channel block cb, tap, half s): the halo rows shifted by the tap; a 16-row block
  // step keeps (row & 7), so one swizzled base serves every block (+ 2 KiB each). A lane whose
  // shifted row leaves its sequence reads the zero slot instead (address select: no wait for the
  // data, no branch -- a branch here makes hipcc drain every outstanding read at the join).
  auto read_g1 = [&](int cb, int tap, int s, int slot, FragsT<MB> &f) {
    if (FFN_ABLATE & 4) return;
    read_a(slot, f);
    const bool all_ok = ((need_mask >> tap) & 1u) == 0;
    const int sh = tap - pad;
    const int hr = hrow0 + tap;
    const int hb = H_OFF + (cb & 1) * HALO_BYTES + hr * 128 + (((s * 4 + (lane >> 4)) ^ (hr & 7)) << 4);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const bool ok = all_ok || (unsigned)(tpos[mb] + sh) < (unsigned)tlen[mb];
      f.b[mb] = *reinterpret_cast<const bf16x8 *>(smem + (ok ? hb + mb * 2048 : ZERO_OFF));
    }
  };
  // GEMM2 unit q (32 hidden columns of the chunk): H column block q / 2, half q % 2
  auto read_g2 = [&](int q, int slot, FragsT<MB> &f) {
    if (FFN_ABLATE & 4) return;
    read_a(slot, f);
    const char *hp = smem + H_OFF + (q >> 1) * H_BLK + hrow0 * 128 + ((((q & 1) * 4 + (lane >> 4)) ^ (lane & 7)) << 4);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) f.b[mb] = *reinterpret_cast<const bf16x8 *>(hp + mb * 2048);
  };

  f32x4 acc1[4][MB], acc2[4][MB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  auto mma = [&](f32x4 (&acc)[4][MB], const FragsT<MB> &f) {
    if (FFN_ABLATE & 1) return;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[jb], f.b[mb], acc[jb][mb], 0, 0, 0);
  };
  auto bar = []() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // chunk c's hidden slice: H[m][j] = bf16(relu(acc1 + b1)); lane holds 4 consecutive j of row m,
  // all inside column block w
  auto write_h = [&](int c) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int jj = jb * 16 + 4 * (lane >> 4);  // column inside block w
      const float4 bb = *reinterpret_cast<const float4 *>(smem + B1_OFF + 4 * (c * kChunk + w * 64 + jj));
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const f32x4 v = acc1[jb][mb];
        bf16x4 o;
        o[0] = (bf16)fmaxf(v[0] + bb.x, 0.f);
        o[1] = (bf16)fmaxf(v[1] + bb.y, 0.f);
        o[2] = (bf16)fmaxf(v[2] + bb.z, 0.f);
        o[3] = (bf16)fmaxf(v[3] + bb.w, 0.f);
        const int m = hrow0 + mb * 16;
        *reinterpret_cast<bf16x4 *>(smem + H_OFF + w * H_BLK + m * 128 + (((jj >> 3) ^ (lane & 7)) << 4) +
                                    (jj & 7) * 2) = o;
        acc1[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  // ---- prologue: halo 0 + halo 1 (both buffers free), units 0 .. NU-2 of this wave's ring
  issue_halo(0, 0);
  issue_halo(1, 1);
  int pc = 0, pp = 0, ph = 0;  // producer: chunk, pair, half of the unit issued next
  auto produce = [&](int slot) {
    issue_unit(pc, pp, ph, slot);
    if (++ph == 2) {
      ph = 0;
      if (++pp == NPC) {
        pp = 0;
        ++pc;
      }
    }
  };
#pragma unroll
  for (int u = 0; u < kNU - 1; ++u) produce(u);
  // halos 0 / 1 and unit 0 landed (units 1 .. NU-2 may stay in flight), every wave's pieces
  // visible; b1 stored
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  bar();
  FragsT<MB> f0, f1;
  read_g1(0, 0, 0, 0, f0);
  int sread = 1;           // ring slot of the next unit to read (unit u + 1)
  int sprod = kNU - 1;     // ring slot the producer fills next (unit u + NU - 1)

  // One iteration = unit u (its fragments fc were read by the previous iteration): wait for this
  // wave's own unit u + 1 (vmcnt(12): units u + 2 .. u + 4 may stay in flight; a halo issued in
  // the last three iterations only makes it wait longer), refill the slot of unit u - 1 (its
  // fragments are in registers) with unit u + 5, read unit u + 1 into fn, then the 28 MFMAs of
  // unit u: the LDS reads of u + 1 overlap the matrix work of u. No barrier: the ring is private.
  auto iter = [&](f32x4 (&acc)[4][MB], FragsT<MB> &fc, auto &&pre, auto &&rd) {
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    pre();
    produce(sprod);
    sprod = sprod == kNU - 1 ? 0 : sprod + 1;
    rd(sread);
    sread = sread == kNU - 1 ? 0 : sread + 1;
    mma(acc, fc);
  };
  // the units of a shared-data hand-off (inside `pre`, after the iteration's waits): every wave's
  // halo / H writes visible, every wave past its reads of the buffer about to be refilled
  auto nopre = [] {};
  // Units alternate f0 / f1 (even units read theirs from f0; a chunk has an even number of units).
  // Every iter() call site is unconditional: a call inside a branch makes hipcc merge the
  // accumulators through a phi and copy all 112 of them every unit.
#pragma nounroll
  for (int c = 0; c < NCH; ++c) {
#pragma nounroll
    for (int cb = 0; cb < 4; ++cb) {
#pragma nounroll
      for (int tap = 0; tap < KS; ++tap) {
        iter(acc1, f0, nopre, [&](int sl) { read_g1(cb, tap, 1, sl, f1); });
        // after the last tap of block cb: the next block's halo becomes visible to every wave (the
        // barrier), and every wave is past its reads of block cb (its last unit is in registers),
        // whose buffer takes block cb + 2 (issued by all waves, consumed 2*KS units later)
        const bool last_tap = tap + 1 == KS;
        iter(acc1, f1,
             [&] {
               if (last_tap && cb + 1 < 4) {
                 bar();
                 if (cb + 2 < 4) issue_halo(cb + 2, cb & 1);
               }
             },
             [&](int sl) {
               if (!last_tap)
                 read_g1(cb, tap + 1, 0, sl, f0);
               else if (cb + 1 < 4)
                 read_g1(cb + 1, 0, 0, sl, f0);
               // (after the last GEMM1 unit the next unit reads H: below)
             });
      }
    }
    // every wave is past its halo reads (barrier): H overwrites the halo buffers; then H visible
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    bar();
    write_h(c);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    bar();
    // (the last GEMM1 iteration advanced sread past this unit without reading it)
    read_g2(0, sread == 0 ? kNU - 1 : sread - 1, f0);
#pragma nounroll
    for (int q = 0; q < kChunk / 32; q += 2) {
      const bool more = c + 1 < NCH, last = q + 2 == kChunk / 32;
      // at unit 4: every wave is past its reads of H blocks 0-1 (units 0..3): the next chunk's
      // first halo goes there
      iter(acc2, f0,
           [&] {
             if (q == 4 && more) {
               bar();
               issue_halo(0, 0);
             }
           },
           [&](int sl) { read_g2(q + 1, sl, f1); });
      // at the last unit: every wave is past its H reads: the next chunk's second halo into H
      // blocks 1-2; its first halo (issued 3 units ago) is visible after the barrier
      iter(acc2, f1,
           [&] {
             if (last && more) {
               bar();
               issue_halo(1, 1);
             }
           },
           [&](int sl) {
             if (!last)
               read_g2(q + 2, sl, f0);
             else if (more)
               read_g1(0, 0, 0, sl, f0);
           });
    }
  }

  // ---- LN epilogue: Y^T accumulators -> E[m][n] f32 -> conv_common.h epilogue (RES_LN)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  bar();  // every wave is past its last LDS read: E may overwrite the rings / H
  float *E = reinterpret_cast<float *>(smem);
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      *reinterpret_cast<f32x4 *>(E + (hrow0 + mb * 16) * EPI_LD + w * 64 + nb * 16 + 4 * (lane >> 4)) =
          acc2[nb][mb];
  __syncthreads();
  epilogue<BM, 256, 4, true>(a, E, m0, 0, tid, M);
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
  const int64_t M64 = (int64_t)d->B * d->T;
  if (M64 > 0x7fffff00LL) return FS2_EINVAL;
  if (M64 == 0) return FS2_OK;
  const int64_t xb = M64 * d->x_row_stride * 2;
  const int64_t wb = (int64_t)(d->F + kD) * fs2_ffn_pitch(d->KS, d->F) * 2;
  if (xb >= (1LL << 31)) return FS2_EUNSUPPORTED;

  FfnArgs p;
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
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  p.w = reinterpret_cast<const bf16 *>(d->w);
  p.b1 = d->b1;
  p.w_bytes = (uint32_t)wb;
  constexpr int BM = 112;
  const int nwg = (int)((M64 + BM - 1) / BM);
  const int nch = d->F / kChunk;
  hipStream_t s = as_stream(stream);
  // instantiated shapes: kernel 9 (model.yaml conv_kernel_size [9, 1]) or 3, F = 1024 or 512
  if (d->KS == 9 && nch == 4)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 9, 4>), dim3(nwg), dim3(256), 0, s, p);
  else if (d->KS == 9 && nch == 2)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 9, 2>), dim3(nwg), dim3(256), 0, s, p);
  else if (d->KS == 3 && nch == 4)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 3, 4>), dim3(nwg), dim3(256), 0, s, p);
  else if (d->KS == 3 && nch == 2)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 3, 2>), dim3(nwg), dim3(256), 0, s, p);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_ffn_pitch(int KS, int F) { return ffn_pitch(KS, F); }
