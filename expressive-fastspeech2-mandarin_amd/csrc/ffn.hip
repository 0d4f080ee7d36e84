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
// the B side (columns m), so every k-step streams one 16 KiB weight stage: 256 weight rows x 32
// channels (64 B per row). 8 waves = 2 (M halves: 64 + 48 rows) x 4 (weight-row quarters of 64);
// waves w and w + 4 share a SIMD, so every SIMD carries 7 of the 112 rows' 16-row blocks.
//
// Pipeline: one k-step per iteration, NS = 4 LDS-DMA stages (3 in flight), one counted vmcnt and
// one raw s_barrier per step; each wave reads the NEXT step's fragments right after the barrier
// and issues this step's MFMAs behind them (two fragment register sets). The x rows of a 64-channel
// block (the tile + the taps' halo, 120 x 128 B) are DMA'd once per (chunk, block) into a 2-deep
// halo ring and read shifted by the tap; a fragment whose shifted row leaves its sequence is zeroed
// (waves whose rows all lie inside one sequence skip the test). LDS: ring 64 KiB + halo 32 KiB +
// H 56 KiB + b1 4 KiB = 156 KiB, one workgroup per CU; the LN epilogue reuses it.
#include <type_traits>

#include "conv_common.h"
#include "fs2_common.h"

namespace {

constexpr int kD = 256;          // d_model (encoder_hidden / decoder_hidden)
constexpr int kChunk = 256;      // hidden columns per chunk
constexpr int kNS = 4;           // weight stages in the ring
constexpr int kStage = 256 * 64; // one stage: 256 weight rows x 32 bf16 channels

struct FfnArgs {
  ConvArgs e;          // x / rows / LN epilogue fields (conv_common.h); e.w unused
  const bf16 *w;       // fs2_ffn_desc.w: F rows of W1 ([KS][256]) then 256 rows of W2 ([F]), pitch ffn_pitch
  const float *b1;     // [F]
  uint32_t w_bytes;
};

// row pitch (elements) of the packed FFN weights: one pitch for both matrices, so a weight stage
// row of either GEMM is the same lane offset (only the scalar stage offset differs)
constexpr int ffn_pitch(int KS, int F) { return KS * 256 > F ? KS * 256 : F; }

// physical 16-byte chunk of logical chunk c (0..3) in a 64-byte stage row r: rows r and r + 8
// swap chunk pairs, which makes the 16-row fragment reads (ds_read_b128 lane groups) conflict-free
__device__ __forceinline__ int stage_chunk(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

template <int MB>
struct FragsT {
  bf16x8 a[4];   // weight rows: 4 blocks of 16
  bf16x8 b[MB];  // activation rows: MB blocks of 16
};

template <int HB, int KS, int NCH>
__global__ __launch_bounds__(512, 1) void ffn_fused_kernel(FfnArgs p) {
  constexpr int BM = 16 * HB;
  static_assert(HB > 4 && HB <= 8, "two M halves: 4 + (HB - 4) blocks");
  constexpr int HALO_PIECES = (BM + 8 + 7) / 8;     // 8-row pieces of one 64-channel halo
  constexpr int APW = (HALO_PIECES + 7) / 8;        // halo pieces per wave (every wave issues APW)
  constexpr int HALO_BYTES = APW * 8 * 1024;
  constexpr int RING_OFF = 0, HALO_OFF = kNS * kStage;
  constexpr int H_OFF = HALO_OFF + 2 * HALO_BYTES;
  constexpr int B1_OFF = H_OFF + BM * 512;
  constexpr int EPI_LD = 256 + 4;
  constexpr int SMEM0 = B1_OFF + 4096;
  constexpr int SMEM = SMEM0 > BM * EPI_LD * 4 ? SMEM0 : BM * EPI_LD * 4;
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const ConvArgs &a = p.e;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;        // M half, weight-row quarter
  const int MBr = wm == 0 ? 4 : HB - 4;     // 16-row blocks of this wave's M half
  const int M = a.rows_dev != nullptr ? *a.rows_dev : a.M;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int pad = a.pad, T = a.T;
  constexpr int F = NCH * kChunk;
  constexpr int NHALO = NCH * 4;
  static_assert((kNS & (kNS - 1)) == 0, "ring slots: power of two");

  // ---- b1 -> LDS (plain loads before any LDS-DMA is in flight)
  for (int i = tid; i < F / 4; i += 512)
    *reinterpret_cast<float4 *>(smem + B1_OFF + 16 * i) = reinterpret_cast<const float4 *>(p.b1)[i];

  // ---- tap validity of this lane's activation rows (sequence position / length)
  int tpos[4], tlen[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = m0 + wm * 64 + mb * 16 + (lane & 15);
    if (mb >= MBr || m >= M) {
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
  const int WR = 16 * MBr, mw = m0 + wm * 64;
  int tw = 0, lw = 0;
  if (mw < M) {
    if (a.row_pos != nullptr) {
      const int2 q = a.row_pos[mw];
      tw = q.x;
      lw = q.y;
    } else {
      tw = mw % T;
      lw = T;
    }
  }
  const bool wave_inside = tw + WR <= lw && mw + WR <= M;
  // taps whose shifted rows may leave a sequence for this wave (bit tap): their fragments are masked
  uint32_t need_mask = 0;
#pragma unroll
  for (int tap = 0; tap < KS; ++tap) {
    const int sh = tap - a.pad;
    if (!(wave_inside && tw + sh >= 0 && tw + WR - 1 + sh < lw)) need_mask |= 1u << tap;
  }
  // consume the row_pos loads here: a first use behind the LDS-DMA stream would drain it
  asm volatile("" ::"v"(tpos[0]), "v"(tpos[1]), "v"(tpos[2]), "v"(tpos[3]), "v"(tlen[0]), "v"(tlen[1]), "v"(tlen[2]),
               "v"(tlen[3]), "v"(tw), "v"(lw));

  // ---- DMA addressing
  constexpr int PITCH = ffn_pitch(KS, F);
  constexpr uint32_t wrow = (uint32_t)PITCH * 2u, w2off = (uint32_t)F * wrow;
  const rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  const uint32_t xrow = (uint32_t)a.xs * 2u;
  // this lane's part of its two stage pieces: weight rows sr0 / sr0 + 16, its 16-byte chunk
  const uint32_t sr0 = (uint32_t)(32 * w + (lane >> 2));
  const uint32_t lo0 = sr0 * wrow + (uint32_t)stage_chunk(sr0, lane & 3) * 16u;
  const uint32_t lo1 = (sr0 + 16) * wrow + (uint32_t)stage_chunk(sr0 + 16, lane & 3) * 16u;
  auto glds = [&](rsrc_t rs, char *dst, uint32_t off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)dst, 16, off, 0, 0, 0);
  };
  // Weight-stage schedule. A "pair" is one 64-channel k-step = two 32-channel stages (+64 B apart
  // in both GEMMs). Pairs of a chunk: GEMM1 pr = cb * KS + tap (pr < NP1), then GEMM2 pr = NP1 + qp
  // (64 hidden columns). Lane pr of ptab_off / ptab_str holds pair pr's byte offset in chunk 0
  // and the chunk stride: the producer reads both with v_readlane instead of decoding the step
  // (every wave runs its scalar code, and a SIMD's two waves share one scalar issue slot).
  constexpr int NP1 = 4 * KS, NPC = NP1 + kChunk / 64;
  static_assert(NPC <= 64, "one table lane per pair");
  const int tl = lane < NPC ? lane : NPC - 1;
  const uint32_t ptab_off = tl < NP1 ? (uint32_t)((tl % KS) * (2 * kD) + (tl / KS) * 128)
                                     : w2off + (uint32_t)(128 * (tl - NP1));
  const uint32_t ptab_str = tl < NP1 ? (uint32_t)kChunk * wrow : (uint32_t)(2 * kChunk);
  // stage `half` of pair (c, pr) into ring slot `slot`. Past the last pair (c == NCH) the offsets
  // run into W2 or past the buffer (zeros): harmless loads that keep every step's vmcnt count equal.
  auto issue_stage = [&](int c, int pr, int half, int slot) {
    const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)ptab_off, pr) +
                         (uint32_t)c * (uint32_t)__builtin_amdgcn_readlane((int)ptab_str, pr) + (uint32_t)(half * 64);
    char *dst = smem + RING_OFF + slot * kStage + 2 * w * 1024;
    glds(wr, dst, lo0 + off);
    glds(wr, dst + 1024, lo1 + off);
  };
  // halo h = chunk * 4 + channel block: rows m0 - pad .. m0 + BM + KS - 2, 128 B (64 channels) each
  const int prow = lane >> 3, plc = (lane & 7) ^ ((lane >> 3) & 7);
  auto issue_halo = [&](int h) {
    const int cb = h & 3;
    char *dst = smem + HALO_OFF + (h & 1) * HALO_BYTES;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int pc = w + 8 * i;
      const int hr = 8 * pc + prow;
      const int gm = m0 - pad + hr;
      const bool ok = hr < BM + KS - 1 && gm >= 0 && gm < M;
      glds(xr, dst + pc * 1024, ok ? (uint32_t)gm * xrow + (uint32_t)(cb * 64 + plc * 8) * 2u : kOOB);
    }
  };

  // The main loop, compiled per M-half size (4 or HB - 4 blocks of 16 rows): exact accumulator
  // and fragment arrays, no per-block guards.
  auto run = [&](auto mbc) {
    constexpr int MB = decltype(mbc)::value;
    // ---- fragment addressing
    const int aoff = (wn * 64 + (lane & 15)) * 64 + stage_chunk(lane & 15, lane >> 4) * 16;
    const int hrow0 = wm * 64 + (lane & 15);  // activation row (tile-relative) of block 0
    auto read_a = [&](int slot, FragsT<MB> &f) {
      const char *st = smem + RING_OFF + slot * kStage + aoff;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) f.a[jb] = *reinterpret_cast<const bf16x8 *>(st + jb * 1024);
    };
    // GEMM1 step (channel block cb, tap, half hs): the halo rows shifted by the tap; a 16-row block
    // step keeps (row & 7), so one swizzled base serves every block (+ 2 KiB each)
    auto read_g1 = [&](int cb, int tap, int hs, int slot, FragsT<MB> &f) {
      read_a(slot, f);
      const int hr = hrow0 + tap;
      const char *hb = smem + HALO_OFF + (cb & 1) * HALO_BYTES + hr * 128 + (((hs * 4 + (lane >> 4)) ^ (hr & 7)) << 4);
      const int sh = tap - pad;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) f.b[mb] = *reinterpret_cast<const bf16x8 *>(hb + mb * 2048);
      if ((need_mask >> tap) & 1u) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          if ((unsigned)(tpos[mb] + sh) >= (unsigned)tlen[mb]) f.b[mb] = bf16x8{};
      }
    };
    // GEMM2 step q (32 hidden columns of the chunk): rows of H
    auto read_g2 = [&](int q, int slot, FragsT<MB> &f) {
      read_a(slot, f);
      const char *hp = smem + H_OFF + hrow0 * 512 + (((4 * q + (lane >> 4)) ^ (lane & 15)) << 4);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) f.b[mb] = *reinterpret_cast<const bf16x8 *>(hp + mb * 16 * 512);
    };

    f32x4 acc1[4][MB], acc2[4][MB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+v"(acc1[i][j]), "+v"(acc2[i][j]));  // no zero-accumulator peeling
      }
    auto mma = [&](f32x4 (&acc)[4][MB], const FragsT<MB> &f) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
            acc[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[jb], f.b[mb], acc[jb][mb], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    auto bar = []() {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto lgkm0 = []() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

    // chunk c's hidden slice: H[m][j] = bf16(relu(acc1 + b1)), lane holds 4 consecutive j of row m
    auto write_h = [&](int c) {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int j = wn * 64 + jb * 16 + 4 * (lane >> 4);
        const float4 bb = *reinterpret_cast<const float4 *>(smem + B1_OFF + 4 * (c * kChunk + j));
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          {
            const f32x4 v = acc1[jb][mb];
            bf16x4 o;
            o[0] = (bf16)fmaxf(v[0] + bb.x, 0.f);
            o[1] = (bf16)fmaxf(v[1] + bb.y, 0.f);
            o[2] = (bf16)fmaxf(v[2] + bb.z, 0.f);
            o[3] = (bf16)fmaxf(v[3] + bb.w, 0.f);
            const int m = hrow0 + mb * 16;
            *reinterpret_cast<bf16x4 *>(smem + H_OFF + m * 512 + (((j >> 3) ^ (lane & 15)) << 4) + (j & 7) * 2) = o;
          }
          acc1[jb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    };

    // ---- prologue: halo 0, stages 0 .. NS-1 (pairs 0, 1); wait for halo 0 + stage 0
    issue_halo(0);
#pragma unroll
    for (int i = 0; i < kNS; ++i) issue_stage(0, i >> 1, i & 1, i);
    int pc = 0, pp = kNS / 2;  // producer: chunk, pair (the pair whose stages are issued next)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // 3 stages x 2 pieces may stay in flight
    lgkm0();  // b1 copy
    bar();
    FragsT<MB> f0, f1;
    read_g1(0, 0, 0, 0, f0);

    // One step t: wait for stage t + 1 (vmcnt(4): the 2 youngest stages, 2 pieces each, may stay
    // in flight; a halo issued in the last two steps makes it wait one stage early, once per 2*KS
    // steps), barrier, this step's MFMAs (fragments in fc), then stage t + NS into the slot step
    // t's fragments came from and the next step's fragment reads (`rd`).
    auto step = [&](auto half, int t, f32x4 (&acc)[4][MB], FragsT<MB> &fc, auto &&rd) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      lgkm0();
      bar();
      // MFMAs first (their operands are in registers): the DMA issue and the fragment reads of the
      // next step go out behind them while the matrix pipe works
      mma(acc, fc);
      issue_stage(pc, pp, decltype(half)::value, t & (kNS - 1));
      if constexpr (decltype(half)::value == 1) {
        if (++pp == NPC) {
          pp = 0;
          ++pc;
        }
      }
      rd();
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    int t = 0;  // global step: ring slot t & (NS - 1); even steps hold fragments in f0
#pragma nounroll
    for (int c = 0; c < NCH; ++c) {
#pragma nounroll
      for (int cb = 0; cb < 4; ++cb) {
#pragma nounroll
        for (int tap = 0; tap < KS; ++tap, t += 2) {
          // the first step of halo h = 4c + cb issues halo h + 1 (into the buffer of halo h - 1,
          // whose last fragments were read before this step's barrier)
          step(H0{}, t, acc1, f0, [&] {
            if (tap == 0 && c * 4 + cb + 1 < NHALO) issue_halo(c * 4 + cb + 1);
            read_g1(cb, tap, 1, (t + 1) & (kNS - 1), f1);
          });
          step(H1{}, t + 1, acc1, f1, [&] {
            if (tap + 1 < KS)
              read_g1(cb, tap + 1, 0, (t + 2) & (kNS - 1), f0);
            else if (cb + 1 < 4)
              read_g1(cb + 1, 0, 0, (t + 2) & (kNS - 1), f0);
            // (after the last GEMM1 step the next fragments need H: read below)
          });
        }
      }
      write_h(c);
      lgkm0();
      bar();
      read_g2(0, t & (kNS - 1), f0);
#pragma nounroll
      for (int qp = 0; qp < kChunk / 64; ++qp, t += 2) {
        step(H0{}, t, acc2, f0, [&] { read_g2(2 * qp + 1, (t + 1) & (kNS - 1), f1); });
        step(H1{}, t + 1, acc2, f1, [&] {
          if (2 * qp + 2 < kChunk / 32)
            read_g2(2 * qp + 2, (t + 2) & (kNS - 1), f0);
          else if (c + 1 < NCH)
            read_g1(0, 0, 0, (t + 2) & (kNS - 1), f0);
        });
      }
    }

    // ---- LN epilogue: Y^T accumulators -> E[m][n] f32 -> conv_common.h epilogue (RES_LN)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bar();  // every wave is past its last LDS read: E may overwrite the ring / halo / H
    float *E = reinterpret_cast<float *>(smem);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        *reinterpret_cast<f32x4 *>(E + (hrow0 + mb * 16) * EPI_LD + wn * 64 + nb * 16 + 4 * (lane >> 4)) =
              acc2[nb][mb];
  };
  if (wm == 0)
    run(std::integral_constant<int, 4>{});
  else
    run(std::integral_constant<int, HB - 4>{});
  __syncthreads();
  epilogue<BM, 256, 8, true>(a, reinterpret_cast<const float *>(smem), m0, 0, tid, M);
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
    hipLaunchKernelGGL((ffn_fused_kernel<7, 9, 4>), dim3(nwg), dim3(512), 0, s, p);
  else if (d->KS == 9 && nch == 2)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 9, 2>), dim3(nwg), dim3(512), 0, s, p);
  else if (d->KS == 3 && nch == 4)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 3, 4>), dim3(nwg), dim3(512), 0, s, p);
  else if (d->KS == 3 && nch == 2)
    hipLaunchKernelGGL((ffn_fused_kernel<7, 3, 2>), dim3(nwg), dim3(512), 0, s, p);
  else
    return FS2_EUNSUPPORTED;
  FS2_CHECK_LAUNCH();
  return FS2_OK;
}

extern "C" int fs2_ffn_pitch(int KS, int F) { return ffn_pitch(KS, F); }
