/*
 * fs2hip.h — C ABI of libfs2hip.so, the MI355X (gfx950 / CDNA4) kernels of the FastSpeech2
 * mel-synthesis forward (Napoliee/Expressive-FastSpeech2-Mandarin).
 *
 * Plain pointers and sizes only: every pointer is a device pointer the caller allocated
 * (HBM), every launch goes on the caller's stream, nothing is allocated or synchronised
 * inside, and there is no global mutable state (reentrant; one call per DataParallel
 * thread is fine). Return value: 0 (FS2_OK) or an fs2_status code; the Python host layer
 * (fs2amd/_lib.py) maps non-zero codes to RuntimeError.
 *
 * Layouts: activations are row-major [B, T, C] ("rows" = (b, t) pairs, C contiguous; a
 * row stride in ELEMENTS may exceed C). dtype codes: FS2_F32 / FS2_BF16.
 * Reference citations are /root/reference paths (the reference is pure PyTorch: these
 * entry points replace the implicit ATen kernels its modules dispatch).
 */
#ifndef FS2HIP_H
#define FS2HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *fs2_stream_t; /* a hipStream_t (NULL = default stream) */

enum fs2_dtype { FS2_F32 = 0, FS2_BF16 = 1, FS2_FP8 = 2 /* OCP e4m3fn bytes (gfx950 MFMA format) */ };

enum fs2_status {
  FS2_OK = 0,
  FS2_EINVAL = 1,       /* bad argument / shape the kernels do not cover */
  FS2_ELAUNCH = 2,      /* hipGetLastError() after the launch was non-zero */
  FS2_EUNSUPPORTED = 3, /* dtype / tile combination not instantiated */
};

/* ---- epilogues of fs2_conv1d ------------------------------------------------------------ */
enum fs2_epilogue {
  FS2_EPI_BIAS = 0,        /* y = acc + bias                                                */
  FS2_EPI_BIAS_RELU = 1,   /* y = relu(acc + bias)            (FFN w_1, SubLayers.py:88)    */
  FS2_EPI_BIAS_TANH = 2,   /* y = tanh(acc + bias)            (PostNet, Layers.py:133)      */
  FS2_EPI_BIAS_RES = 3,    /* y = acc + bias + residual       (PostNet residual, fastspeech2.py:136) */
  FS2_EPI_RES_LN = 4,      /* y = LN(acc + bias + residual); rows t >= lens[b] -> 0;
                              then y += addvec1[b] (+ addvec2[b]).  Requires N == 256.
                              (MHA fc / FFN w_2 + LayerNorm + masked_fill, SubLayers.py:54-55,
                              :88-91, Layers.py:25,28; speaker/emotion add fastspeech2.py:101-110) */
  FS2_EPI_RELU_LN = 5,     /* y = LN(relu(acc + bias))        (VariancePredictor, modules.py:218-233) */
  FS2_EPI_RELU_LN_DOT = 6, /* out[row] = (t >= lens[b]) ? 0 : dot(LN(relu(acc+bias)), dot_w) + dot_b
                              -> f32 [B*T]                    (VP linear + masked_fill, modules.py:240-250) */
  FS2_EPI_BIAS_LRELU = 7,  /* y = leaky_relu(acc + bias, act_slope)
                              (HiFi-GAN ResBlock convs1 + the leaky_relu before convs2, hifigan/models.py:101-104) */
  FS2_EPI_RES_SUM = 8,     /* y = (acc + bias + residual [+ residual2]) / out_div
                              (ResBlock residual x = xt + x :104; the multi-receptive-field sum
                              xs += resblock(x), x = xs / num_kernels, hifigan/models.py:152-158) */
  FS2_EPI_RELU_GRAD = 9,   /* y = (residual > 0) ? acc + bias : 0
                              (training backward through the FFN's relu, SubLayers.py:88: the
                              input gradient of w_2 masked by the saved relu output)           */
};

/*
 * fs2_conv1d — implicit-GEMM Conv1d / Linear over padded sequences, bf16 or f32 MFMA.
 *
 *   y[b,t,n] = epi( sum_{k<KS} sum_{c<Cin} x[b, t+k-pad, c] * w[n][k][c] + bias[n] )
 *
 * with x[b, s, :] = 0 outside s in [0, T) (per-sequence zero padding, as nn.Conv1d on the
 * [B, C, T] transpose; padded frames INSIDE [0, T) are read as they are).
 * KS = 1, pad = 0 is nn.Linear.  Replaces: nn.Linear in MultiHeadAttention (w_qs/w_ks/w_vs
 * fused into one N=768 GEMM, fc) transformer/SubLayers.py:18-20,39-41,54; nn.Conv1d in
 * PositionwiseFeedForward SubLayers.py:68-80; VariancePredictor Conv model/modules.py:253-296;
 * mel_linear model/fastspeech2.py:23-26,134; PostNet ConvNorm+BatchNorm1d(eval, folded into
 * w and bias by the host) transformer/Layers.py:33-137.
 *
 * w is PACKED: [N][KS][Cin_pad] in the compute dtype, Cin_pad = Cin rounded up to 64 (bf16)
 * or 32 (f32) with zeros (fs2_conv_cin_pad()). Cin and N must be multiples of 8 and 4.
 *
 * Packed sequences (rows_dev != NULL): x / residual / out hold only the valid frames of each
 * sequence back to back (fs2_seq_layout); the grid is sized for B*T rows (capacity) and the
 * active row count *rows_dev is read on the device, so no host sync is needed. Row r is frame
 * row_pos[2r] of a sequence of row_pos[2r+1] frames; taps outside [0, len) read zeros. The
 * Decoder runs this way (every masked padded frame of an FFT block is dead work,
 * Decoder.forward, transformer/Models.py:139-171, layer loop :164-167). lens / addvec must be
 * NULL with packed rows.
 * a_rowmap (KS == 1, padded output): A row of output row m is x row a_rowmap[m], or zeros when
 * -1 — mel_linear reading the packed decoder output into the padded [B, T, n_mel] contract.
 */
typedef struct fs2_conv_desc {
  const void *x;            /* [B, T, >=Cin], dtype x_dtype                              */
  int x_dtype;
  int64_t x_row_stride;     /* elements between rows of x                                  */
  const void *w;            /* packed weights (compute dtype)                              */
  const float *bias;        /* [N] or NULL                                                 */
  int B, T, Cin, Cin_pad, N, KS, pad;
  int compute;              /* FS2_BF16 (mfma_f32_16x16x32_bf16) or FS2_F32 (mfma_f32_16x16x4f32) */
  int epilogue;             /* enum fs2_epilogue                                           */
  const void *residual;     /* [B, T, N] (BIAS_RES / RES_LN)                               */
  int res_dtype;
  int64_t res_row_stride;
  const float *ln_gamma;    /* [N] (LN epilogues)                                          */
  const float *ln_beta;
  float ln_eps;
  const int64_t *lens;      /* [B] valid rows per sequence (RES_LN / RELU_LN_DOT) or NULL  */
  const float *addvec1;     /* [B, N] or NULL (RES_LN)                                     */
  const float *addvec2;     /* [B, N] or NULL (RES_LN)                                     */
  const float *dot_w;       /* [N] (RELU_LN_DOT)                                           */
  float dot_b;
  void *out;                /* [B, T, N] (f32 [B*T] for RELU_LN_DOT)                       */
  int out_dtype;
  int64_t out_row_stride;
  const int32_t *rows_dev;  /* packed rows: device int32 = active row count, or NULL (padded) */
  const int32_t *row_pos;   /* packed rows: int32 [rows][2] = {frame, sequence length}       */
  const int32_t *a_rowmap;  /* int32 [B*T] packed source row of each output row, or NULL     */
  /* fp8 (compute == FS2_FP8: x and w are e4m3fn bytes, mfma_scale_f32_16x16x128_f8f6f4):        */
  const float *col_scale;   /* [N] dequantisation scale applied to the accumulator before the
                               bias (x scale * per-channel w scale), or NULL                    */
  float out_scale;          /* out_dtype == FS2_FP8: stored value = e4m3(y * out_scale)         */
  void *out2;               /* optional second output, rows of N elements. LN epilogues:
                               e4m3(y * out2_scale) (the fp8 copy the next fp8 GEMM reads);
                               elementwise epilogues: bf16(y) (e.g. mel_linear's f32 output
                               for the residual + its bf16 copy for PostNet's first conv)      */
  float out2_scale;
  /* split-precision (bf16x3) GEMM: the logical input channels are blocks of cin_block channels,
     block i read from source channel cin_src[i] of x (e.g. [x_hi | x_hi | x_lo] against packed
     weights [w_hi | w_lo | w_hi]); 0 = off. LN epilogue: out_split = 1 stores y as two bf16
     planes per row, hi at column n and lo = bf16(y - hi) at column N + n.                    */
  int cin_block;
  int cin_src[4];
  int out_split;
  /* split-K tail workspace (optional, NULL = off): when a launch's tiles leave a small last
     round, its tiles are split along K across the idle workgroups and summed in fixed segment
     order by the last arriving segment. The first 4 KiB are arrival counters and MUST be zero
     before first use (they reset themselves); the rest holds f32 partial tiles. 128 MiB + 4 KiB
     covers 256 CUs (32 MiB + 4 KiB without the phased kernel's stream-K tail). One workspace per stream: concurrent launches must not share it. Results
     are deterministic but not bitwise equal to the unsplit summation order.                  */
  void *splitk_ws;
  int64_t splitk_ws_bytes;
  /* ---- vocoder extensions (HiFi-GAN generator, hifigan/models.py; zero = off / defaults) ---- */
  int dilation;             /* tap k reads x[b, t + k*dilation - pad]; 0 or 1 = undilated. Non-LN
                               epilogues allow KS <= 11 and (KS-1)*dilation + 1 <= 51            */
  float act_slope;          /* FS2_EPI_BIAS_LRELU negative slope                                 */
  int out2_act;             /* elementwise epilogues: 0 = out2 is a copy of y, 1 = leaky_relu(y,
                               out2_slope) (the next layer's leaky_relu fused into this one)     */
  float out2_slope;
  int out2_f32;             /* elementwise epilogues: out2 in f32 instead of bf16                 */
  const void *residual2;    /* FS2_EPI_RES_SUM: optional second addend, out's dtype and row stride
                               (may alias out: each element is read before it is written)        */
  float out_div;            /* FS2_EPI_RES_SUM: divisor applied last (0 = 1)                       */
  /* ---- grouped input (the variance predictors' column-split form; 0 = off) ----
     Output columns [g*group_n, (g+1)*group_n) read the input channels shifted by g*group_cin
     (after the cin_block map): two predictors' conv2 in one launch, each on its own hidden
     planes. Elementwise epilogues only; group_n a multiple of 128.                           */
  int group_n;
  int group_cin;
} fs2_conv_desc;

int fs2_conv1d(const fs2_conv_desc *d, fs2_stream_t stream);
int fs2_conv_cin_pad(int Cin, int compute);

/*
 * fs2_ffn — PositionwiseFeedForward + residual + LayerNorm + padding mask as ONE launch
 * (transformer/SubLayers.py:85-93 w_1 -> ReLU -> w_2 -> dropout(eval) -> LayerNorm(out + residual),
 * then the FFTBlock's masked_fill, transformer/Layers.py:28; speaker/emotion adds as FS2_EPI_RES_LN):
 *
 *   f[m, :] = relu( sum_{k<KS} sum_c x[m + k - pad, c] * w1[j][k][c] + b1[j] )   (per-sequence zero taps)
 *   y[m, :] = LN( f[m, :] . w2^T + b2 + x[m, :] ); rows t >= lens[b] -> 0; y += addvec1[b] (+ addvec2[b])
 *
 * The 1024-wide hidden f never reaches HBM: a workgroup keeps a 112-row tile's f in LDS, one
 * 256-column chunk at a time, and accumulates w_2's product in registers (two fs2_conv1d launches
 * write and re-read it: 51 MB each way per cfg2 decoder block).
 * bf16 only. x / out: bf16 rows of D = 256 (out must not alias x). w: the FFN's two weight
 * matrices in one flat bf16 buffer of fs2_ffn_weight_elems(KS, F) elements, in MFMA fragment
 * order (64-row quads, then k-steps of 32 channels, then 4 blocks of 16 rows, then 64 lanes x 8):
 *   w_1 (Conv1d weight [F][D][KS]) as [F/64][KS][D/32][4][4][16][8], element (q, k, s, b, h, r, e) =
 *       w_1[64q + 16b + r][32s + 8h + e][k];
 *   then w_2 ([D][F][1]) as [D/64][F/32][4][4][16][8], element (q, s, b, h, r, e) =
 *       w_2[64q + 16b + r][32s + 8h + e][0].
 * Shapes: D = 256, F in {512, 1024}, KS in {3, 9}, pad <= KS - 1
 * (FS2_EUNSUPPORTED otherwise: the caller runs the two fs2_conv1d launches). Packed rows (rows_dev / row_pos, fs2_seq_layout) or padded [B, T] rows (lens /
 * addvec allowed) as in fs2_conv1d. Deterministic; each output row depends only on its own input
 * rows, so packed and padded launches agree bit for bit.
 */
typedef struct fs2_ffn_desc {
  const void *x;            /* bf16 [B*T, >= D]: the FFN input and the LayerNorm residual        */
  int64_t x_row_stride;
  const void *w;            /* bf16 w_1 | w_2 in fragment order (see above)                       */
  const float *b1;          /* [F]                                                               */
  const float *b2;          /* [D]                                                               */
  int B, T, D, F, KS, pad;
  const float *ln_gamma;    /* [D]                                                               */
  const float *ln_beta;
  float ln_eps;
  const int64_t *lens;      /* [B] or NULL (padded rows only)                                    */
  const float *addvec1;     /* [B, D] or NULL (padded rows only)                                 */
  const float *addvec2;
  void *out;                /* bf16 [B*T, >= D]                                                  */
  int64_t out_row_stride;
  const int32_t *rows_dev;  /* packed rows (fs2_seq_layout cu + B) or NULL                       */
  const int32_t *row_pos;   /* packed rows: int32 [rows][2] = {frame, sequence length}           */
  /* split-hidden form (optional; nsplit 0 or 1 = off): each 112-row tile is run by nsplit in
     {2, 4} workgroups (nsplit <= F/256), split s computing hidden chunks [s*F/(256*nsplit), ...)
     and its partial w_2 product; the last arriving split sums the f32 partials in split order
     (deterministic, not bitwise equal to nsplit = 1) and runs the LayerNorm epilogue. For launches
     with too few tiles to fill the chip (the 4k-row encoder, short free-running decoders).
     splitk_ws: the fs2_conv1d split-K workspace (first 4 KiB zeroed arrival counters, one per
     tile: <= 1024 tiles; then tiles * nsplit * tile_rows KiB of f32 partials).                 */
  int nsplit;
  void *splitk_ws;
  int64_t splitk_ws_bytes;
  int rows_max;             /* packed rows: an upper bound of *rows_dev the caller knows (e.g. from
                               a host read of the lengths; 0 = B*T): the launch covers only
                               min(*rows_dev, rows_max) rows, its grid and workspace are sized
                               from rows_max                                                      */
  int tile_rows;            /* rows per workgroup tile: 0 / 112 (default) or 64 (the split-hidden
                               form of small launches: 4 splits x 64-row tiles fill the chip, and
                               the last arriver loads the other partials in one round trip)       */
  /* the NEXT FFT block's Q|K|V projection fused into the epilogue (optional, wqkv NULL = off):
     qkv_out[m, n] = bf16( sum_c y[m, c] * wqkv[n][c] + bqkv[n] ), n < nqkv (a multiple of 256),
     for every stored row m (transformer/SubLayers.py:39-41 of block i+1, on block i's output).
     wqkv in fragment order [nqkv/64][D/32][4][4][16][8], element (q, s, b, h, r, e) =
     W[64q + 16b + r][32s + 8h + e] (W = [w_qs; w_ks; w_vs], [nqkv][D]).                     */
  const void *wqkv;
  const float *bqkv;
  void *qkv_out;
  int64_t qkv_row_stride;
  int nqkv;
  /* the block's attention output projection + residual + LayerNorm in the PROLOGUE (optional,
     pre_att NULL = off; packed rows, 112-row tiles, nsplit 1, KS = 9, F = 1024): x is then the
     FFT block's input and the FFN input is computed on chip for the tile and its halo rows,
       h = LN1(pre_att . pre_w^T + pre_b + x)        (transformer/SubLayers.py:54-55, Layers.py:25)
     and the FFN's own LayerNorm residual is h. pre_w: fc weight [256][256] in fragment order
     [4][8][4][4][16][8] (as wqkv). Replaces the fc + residual + LN launch of fs2_conv1d.      */
  const void *pre_att;       /* bf16 [B*T, >= 256]: the attention output (heads concatenated)   */
  int64_t pre_att_row_stride;
  const void *pre_w;
  const float *pre_b;        /* [256]                                                           */
  const float *pre_gamma;    /* [256]                                                           */
  const float *pre_beta;
  float pre_eps;
} fs2_ffn_desc;

int fs2_ffn(const fs2_ffn_desc *d, fs2_stream_t stream);
int64_t fs2_ffn_weight_elems(int KS, int F); /* F*KS*256 + 256*F */

/*
 * fs2_ffn_wide — the same PositionwiseFeedForward + residual + LayerNorm + mask (+ addvecs) as
 * fs2_ffn (transformer/SubLayers.py:85-93, Layers.py:27-30), for small row counts (the encoder's
 * B x L_max phoneme rows), as two wide-tile launches: H = relu(conv_k(x) + b1) into `hidden`
 * (bf16 [rows, F], >= rows * F * 2 bytes; rows = B * T, or rows_max for packed launches) on
 * 256-row x 64-column tiles that keep the x tile in LDS for every tap, then the k = 1 conv on
 * 64 x 64 tiles with the LayerNorm finished by the last of each row tile's 4 column quarters (f32
 * pre-norm rows and arrival counters in d->splitk_ws: 4096 + rows * 1024 bytes, rows <= 65536).
 * Same descriptor as fs2_ffn; tile_rows / nsplit are ignored, wqkv and pre_att must be NULL.
 */
int fs2_ffn_wide(const fs2_ffn_desc *d, void *hidden, int64_t hidden_bytes, fs2_stream_t stream);

/*
 * fs2_ffn8 — the fused PositionwiseFeedForward + residual + LayerNorm on e4m3 MFMA (cfg5; the fp8
 * form of fs2_ffn, v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales). Quantisation points
 * and scales of the two-launch fp8 path (fs2_conv1d, FS2_FP8):
 *   f[m, j] = e4m3( relu(sum_{tap,c} x8[m + tap - pad, c] w1q[j][c][tap] * cs1[j] + b1[j]) * inv_sf )
 *   y[m, n] = LN( sum_j f[m, j] w2q[n][j] * cs2[n] + b2[n] + res[m, n] ),  out8 = e4m3(y * out8_scale)
 * Packed rows only (fs2_seq_layout: rows_dev / row_pos), KS = 9, pad = 4, D = 256, F = 1024.
 * w: fs2_ffn8_weight_bytes(KS, F) e4m3 bytes, w1 then w2, each in 8 KiB units of 64 rows x 128 k:
 *   w1: [F/64][KS*2 units (tap, 128-channel step)][4 blocks][2 halves][4 g][16 r][16 e]
 *   w2: [256/64][F/128 units][4 blocks][2 halves][4 g][16 r][16 e]
 *   element (.., b, h, g, r, e) = W[64q + 16b + r][128u + 32g + 16h + e] (W1[j][tap*256 + c]).
 */
typedef struct fs2_ffn8_desc {
  const void *x8;           /* e4m3 [B*T, >= 256]: the FFN input (fc + LN epilogue's fp8 copy)     */
  int64_t x8_row_stride;
  const void *res;          /* bf16 [B*T, >= 256]: the LayerNorm residual (the same h in bf16)     */
  int64_t res_row_stride;
  const void *w;
  const float *cs1;         /* [F] dequantisation of GEMM1 (input scale x per-row weight scale)    */
  const float *b1;          /* [F]                                                                */
  float inv_sf;             /* 1 / the hidden's quantisation scale                                */
  const float *cs2;         /* [D]                                                                */
  const float *b2;
  int B, T, D, F, KS, pad;
  const float *ln_gamma, *ln_beta;
  float ln_eps;
  void *out;                /* bf16 [B*T, >= 256]                                                 */
  int64_t out_row_stride;
  void *out8;               /* optional e4m3 copy of out (the next block's Q|K|V input) or NULL    */
  int64_t out8_row_stride;
  float out8_scale;
  const int32_t *rows_dev;
  const int32_t *row_pos;
  int rows_max;             /* as fs2_ffn                                                         */
} fs2_ffn8_desc;

int fs2_ffn8(const fs2_ffn8_desc *d, fs2_stream_t stream);
int64_t fs2_ffn8_weight_bytes(int KS, int F);

/*
 * fs2_wconv — a PostNet convolution (transformer/Layers.py:92-137: Conv1d(512, 512, k=5, pad=2) +
 * BatchNorm1d (eval: folded into w / bias on the host) + tanh) on padded [B, T] rows:
 *   y[m, n] = tanh( sum_{k<KS} sum_c x[m + k - pad, c] * w[n][c][k] + bias[n] )   (per-sequence zero taps)
 * bf16 x / out (out must not alias x), f32 accumulation and tanh. w with K = (tap, channel) flattened
 * (k = tap * Cin + c, zero-padded to a multiple of 32) in MFMA fragment order [N/64][K/32][4][4][16][8],
 * element (q, s, b, h, r, e) = W[64q + 16b + r][32s + 8h + e], W[n][tap * Cin + c] = w[n][c][tap]
 * (fs2_wconv_weight_elems(KS, Cin, N) elements). Shapes: N = 512, Cin = 512 (the middle convs) or 80
 * (the first), KS = 5, pad <= KS - 1, epilogue FS2_EPI_BIAS_TANH (FS2_EUNSUPPORTED otherwise: use
 * fs2_conv1d).
 */
typedef struct fs2_wconv_desc {
  const void *x;            /* bf16 [B*T, >= Cin]                                                 */
  int64_t x_row_stride;
  const void *w;            /* bf16, fragment order (see above)                                   */
  const float *bias;        /* [N] (BatchNorm folded)                                             */
  int B, T, Cin, N, KS, pad;
  int epilogue;             /* FS2_EPI_BIAS_TANH                                                  */
  void *out;                /* bf16 [B*T, >= N]                                                   */
  int64_t out_row_stride;
  /* optional second conv on the first one's output, in the same launch (the PostNet's layers 0
     and 1: Cin = 80, N = 512, then 512 -> 512, both k = 5, pad 2, tanh): out = tanh(conv(tanh(
     conv(x; w) + bias); w2) + bias2). w2: fs2_wconv_weight_elems(5, 512, 512) elements, NULL = off */
  const void *w2;
  const float *bias2;
  /* w2 with Cin = 512 (N = 512, KS = 5, pad 2, tanh): the PostNet's last two layers in one launch
     (transformer/Layers.py:92-137 layers 3 and 4 + fastspeech2.py:136): out is then f32 [B*T, >= 80]
     = conv(tanh(conv(x; w) + bias); w2) + bias2 + residual, w2 / bias2 / residual as the
     FS2_EPI_BIAS_RES form below; the 512-channel intermediate never leaves the chip */
  /* epilogue FS2_EPI_BIAS_RES (the PostNet's last conv + the residual, fastspeech2.py:136): Cin = 512,
     N = 80, KS = 5, pad 2; out f32 [B*T, >= 80] = conv(x; w) + bias + residual (f32 [B*T, >= 80]);
     w in the k-step-major order [K/32][N/16][4][16][8], element (s, b, h, r, e) = W[16b + r][32s + 8h + e] */
  const float *residual;
  int64_t res_row_stride;
  /* packed rows (fs2_seq_layout / fs2_seq_layout_margin; both NULL = padded [B, T] rows): row r is
     frame row_pos[2r] of a sequence of row_pos[2r+1] frames, taps outside it read zeros; the active
     row count is *rows_dev (device), the grid covers rows_max rows when 0 < rows_max < B*T */
  const int32_t *rows_dev;
  const int32_t *row_pos;
  int rows_max;
} fs2_wconv_desc;

int fs2_wconv(const fs2_wconv_desc *d, fs2_stream_t stream);
int64_t fs2_wconv_weight_elems(int KS, int Cin, int N); /* N*KS*Cin */

/*
 * fs2_attention — ScaledDotProductAttention with a key-padding mask, all heads.
 * Replaces transformer/Modules.py:14-25 (bmm, /temperature, masked_fill(-inf), softmax(dim=2),
 * bmm) and the head split/merge permutes of SubLayers.py:42-52.
 * qkv: [B, T, 3*H*dk] rows (the fused projection's output): Q at column h*dk, K at
 * (H+h)*dk, V at (2H+h)*dk.  out: [B, T, H*dk], head h at column h*dk.
 * Keys t >= key_lens[b] get zero weight; every query row (padded ones included) is computed.
 * A sequence with key_lens[b] == 0 yields zeros (the reference yields NaN rows that its
 * masked_fill then zeroes).  dk must be 128.
 * seq_cu (int32 [B+1], fs2_seq_layout) != NULL: packed rows — sequence b is rows
 * seq_cu[b] .. seq_cu[b+1]-1 of qkv / out (T = capacity bound on its length; key_lens unused).
 * lse (optional, training): f32 [rows][H], the log2-domain log-sum-exp of each query's scaled
 * scores (log2(e)/temperature units; +inf without a valid key) for fs2_attention_bwd.
 */
int fs2_attention(const void *qkv, int dtype, int64_t qkv_row_stride, const int64_t *key_lens, int B, int T,
                  int H, int dk, float temperature, void *out, int64_t out_row_stride, const int32_t *seq_cu,
                  float *lse, fs2_stream_t stream);
/* fs2_attention with the caller's work-shape hint: waves = 8 (256 queries per workgroup: long,
   dense sequences — most of [B, T] valid, T <= 512), 4 (128 queries) or 0 (fs2_attention's
   default, 4). Same results either way (each query's arithmetic does not depend on the grouping).
   split_ws != NULL: the key-split form (packed rows, lse == NULL, 256 < T <= 2048, H <= 16) over
   the work list fs2_attention_items wrote into split_ws for the same seq_cu: a sequence longer
   than 256 keys is cut into 256-key ranges, one workgroup each, merged by the last range of each
   (query tile, head) to finish — a batch of many short and a few long sequences (free-running
   synthesis) is no longer bound by the longest one's single workgroup. Those sequences' outputs
   then differ from the unsplit form by f32 rounding and depend on their own length only (not on
   T); shorter ones are bit-identical. rows_max >= seq_cu[B]; split_ws:
   fs2_attention_split_ws_bytes(B, T, H, rows_max) bytes (fs2_attention_items zeroes its arrival
   counters; each call leaves them zero). */
int fs2_attention_ex(const void *qkv, int dtype, int64_t qkv_row_stride, const int64_t *key_lens, int B, int T,
                     int H, int dk, float temperature, void *out, int64_t out_row_stride, const int32_t *seq_cu,
                     float *lse, int waves, void *split_ws, int64_t split_ws_bytes, int64_t rows_max,
                     fs2_stream_t stream);
int64_t fs2_attention_split_ws_bytes(int B, int T, int H, int64_t rows_max); /* 0: no split form */
/* the key-split work list of a packed layout (one launch; every layer of a stack reuses it) */
int fs2_attention_items(const int32_t *seq_cu, int B, int T, int H, void *split_ws, int64_t split_ws_bytes,
                        int64_t rows_max, fs2_stream_t stream);

/*
 * fs2_enc_attn_block — the encoder FFT block's attention sub-layer as ONE launch (bf16): Q|K|V
 * projection (transformer/SubLayers.py:39-41), 2-head attention with the key-padding mask
 * (Modules.py:14-25), output projection + residual + LayerNorm (SubLayers.py:54-55) and the
 * padded-row mask (Layers.py:25): out[b, t] = t < lens[b] ? LN(fc(attn(x))[b, t] + x[b, t]) : 0.
 * Replaces fs2_conv1d (Q|K|V) + fs2_attention + fs2_conv1d (EPI_RES_LN) for short sequences: one
 * workgroup per utterance, Q|K|V and the attention output kept in LDS.
 * x / out: bf16 [B, L, 256] (out != x); lens int64 [B]; wqkv / wfc: the [768, 256] / [256, 256]
 * weights in MFMA fragment order ([N/64][K/32][4][4][16][8] bf16, fs2amd.ops.pack_frag_rows);
 * bqkv f32 [768], bfc / gamma / beta f32 [256]. H = 2, dk = 128, L <= 64 (else FS2_EUNSUPPORTED).
 * ws (optional, the fs2_conv_desc split-K workspace: 4 KiB of zeroed int32 counters, then
 * >= B * 128 KiB): two workgroups per utterance, one per head, meeting through a write-through
 * hand-off of their f32 fc halves (the counters are left zero); NULL: one workgroup per utterance.
 */
int fs2_enc_attn_block(const void *x, const int64_t *lens, int B, int L, const void *wqkv, const float *bqkv,
                       const void *wfc, const float *bfc, const float *gamma, const float *beta, float eps, int H,
                       int dk, float temperature, void *out, void *ws, int64_t ws_bytes, fs2_stream_t stream);
/*
 * fs2_enc_embed_attn_block — the FIRST encoder block's attention sub-layer with the encoder input
 * built in the same launch (replaces fs2_embed_pe + fs2_length_masks x 2 + fs2_enc_attn_block):
 * x[b, t] = bf16(emb[tokens[b, t]] + pe[t]) exactly as fs2_embed_pe (an id outside [0, vocab):
 * NaN row, *bad_ids += 1), never written to HBM; src_mask[b, t] = t >= lens[b] (bool [B, L]) and,
 * when mel_mask != NULL, mel_mask[b, t] = t >= mel_lens[b] (bool [B, T_mel]) as fs2_length_masks.
 * Other arguments and limits as fs2_enc_attn_block.
 */
typedef struct fs2_cond_desc {  /* the arguments of fs2_cond_vectors (below), B and D implied */
  const int64_t *speakers;
  const float *speaker_table;
  int n_speaker;
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
  float *spk_out, *emo_out;
} fs2_cond_desc;

/* cond != NULL: fs2_cond_vectors' outputs computed by extra workgroups of the same launch (they run
   on the CUs the B utterance workgroups leave idle); d_emo + d_aro + d_val <= 4096 */
int fs2_enc_embed_attn_block(const int64_t *tokens, const float *emb, int vocab, const float *pe, int32_t *bad_ids,
                             const int64_t *lens, int B, int L, const void *wqkv, const float *bqkv, const void *wfc,
                             const float *bfc, const float *gamma, const float *beta, float eps, int H, int dk,
                             float temperature, void *out, uint8_t *src_mask, const int64_t *mel_lens, int T_mel,
                             uint8_t *mel_mask, const fs2_cond_desc *cond, void *ws, int64_t ws_bytes,
                             fs2_stream_t stream);

/*
 * fs2_attention_bwd — gradient of fs2_attention (training; autograd of transformer/Modules.py:14-25
 * and the head split/merge of SubLayers.py:36-52) without any T x T tensor: two flash-style
 * kernels (dQ per 64-query block with the softmax statistics rebuilt from Q and K; dK / dV per
 * 64-key block reading those statistics back).
 * qkv: the forward's input [rows, >= 3*H*dk] (dtype: FS2_BF16 / FS2_F32, also the MFMA operand
 * type); out: the forward's output [rows, >= H*dk] (same dtype); dout: f32 [rows, >= H*dk].
 * dqkv: f32 [rows, >= 3*H*dk] (dQ | dK | dV in the Q | K | V columns; fully written for every
 * row < T of every sequence). Layout as fs2_attention: key_lens (padded [B, T] rows) XOR seq_cu
 * (packed rows). ws: f32 workspace of >= 2*B*T*H floats (softmax statistics). dk must be 128.
 * lse (optional): the forward's saved statistics (fs2_attention's lse); the dQ kernel then skips
 * its statistics pass.
 */
int fs2_attention_bwd(const void *qkv, int dtype, int64_t qkv_row_stride, const void *out, int64_t out_row_stride,
                      const float *dout, int64_t dout_row_stride, const int64_t *key_lens, int B, int T, int H,
                      int dk, float temperature, float *dqkv, int64_t dqkv_row_stride, const int32_t *seq_cu,
                      float *ws, int64_t ws_bytes, const float *lse, fs2_stream_t stream);

/*
 * fs2_cond_bwd — backward of the training forward's conditioning add (fastspeech2.py:101-110):
 * y[b, l] = x[b, l] + spk_out[b] + emo_out[b] with fwd the forward's fs2_cond_vectors arguments
 * (ids, tables, lin_w; emo_out = its relu output, read for the relu mask; spk_out unused).
 * dy [B, L, D] f32. Every gradient ACCUMULATES into its output (zero it for a fresh gradient); a
 * NULL output is skipped; a table row gets the batch entries with its id in batch order (fixed
 * order, deterministic). ids are clamped into their table as fs2_cond_vectors does. The gradient
 * of x is dy itself (the caller passes it on). ws: fs2_cond_bwd_ws_bytes(B, D) bytes. Needs
 * B <= 64 and, with the emotion path, (B * D + 16 * D + 32 * B) * 4 + 24 * B <= 64 KiB
 * (FS2_EUNSUPPORTED otherwise). Two launches.
 * Replaces the autograd of the three adds, the four nn.Embedding lookups, the cat and
 * emotion_linear (nn.Linear + ReLU) in training.
 */
typedef struct fs2_cond_grads {
  float *d_speaker_table; /* [n_speaker, D] */
  float *d_emo_table;     /* [n_emo, d_emo] */
  float *d_aro_table;     /* [n_aro, d_aro] */
  float *d_val_table;     /* [n_val, d_val] */
  float *d_lin_w;         /* [D, d_emo + d_aro + d_val] */
  float *d_lin_b;         /* [D] */
} fs2_cond_grads;
int64_t fs2_cond_bwd_ws_bytes(int B, int D);
int fs2_cond_bwd(const float *dy, int B, int L, int D, const fs2_cond_desc *fwd, const fs2_cond_grads *grads,
                 void *ws, int64_t ws_bytes, fs2_stream_t stream);

/*
 * fs2_embed_pe — out[b,l,:] = table[tokens[b,l], :] + pe[l, :]   (f32 math)
 * Replaces Encoder src_word_emb + position_enc (transformer/Models.py:82-91).
 * A token outside [0, vocab) — the reference's nn.Embedding raises IndexError (CPU) or a
 * device-side assert (GPU) — makes its output row NaN and adds 1 to *bad_ids (optional int32
 * device counter; the Python layer raises IndexError when it reads a non-zero count).
 */
int fs2_embed_pe(const int64_t *tokens, const float *table, int vocab, const float *pe, int B, int L, int D,
                 void *out, int out_dtype, int32_t *bad_ids, fs2_stream_t stream);

/*
 * fs2_cond_vectors — the per-utterance conditioning vectors added to every encoder position:
 *   spk_out[b] = speaker_table[speakers[b]]                               (fastspeech2.py:101-104)
 *   emo_out[b] = relu(W @ cat(emo[e_b], aro[a_b], val[v_b]) + bias)      (fastspeech2.py:106-110)
 * W is [D][d_emo + d_aro + d_val] (nn.Linear layout).  Either table may be NULL (skipped).
 */
int fs2_cond_vectors(const int64_t *speakers, const float *speaker_table, int n_speaker, const int64_t *emotions,
                     const float *emo_table, int n_emo, int d_emo, const int64_t *arousals, const float *aro_table,
                     int n_aro, int d_aro, const int64_t *valences, const float *val_table, int n_val, int d_val,
                     const float *lin_w, const float *lin_b, int B, int D, float *spk_out, float *emo_out,
                     fs2_stream_t stream);

/*
 * fs2_variance_embed — pitch/energy bucketize + embedding add (model/modules.py:80-100,117-126):
 *   v = target ? target[m] : (pred[m] *= control);  idx = #{bins[i] < v}  (torch.bucketize, right=False)
 *   x[m, :] += table[idx, :]
 * x: [M, D] in place (dtype x_dtype); pred f32 [M] (scaled in place when target == NULL);
 * bins f32 [n_bins - 1]; table f32 [n_bins, D].
 */
int fs2_variance_embed(void *x, int x_dtype, float *pred, const float *target, float control, const float *bins,
                       int n_bins, const float *table, int M, int D, fs2_stream_t stream);
/*
 * fs2_variance_embed_ex — the same bucketize + embedding add, out of place, for training
 *   (model/modules.py:80-100 + VarianceAdaptor.forward :117-126 under autograd):
 *   idx_out[m] = #{bins[i] < value[m]};  out[m, :] = x[m, :] + table[idx_out[m], :]
 * value f32 [M] (the target, or the prediction already scaled by the control); idx_out int64 [M]
 * (optional: the embedding backward's indices, fs2_embedding_bwd).
 */
int fs2_variance_embed_ex(const void *x, int x_dtype, const float *value, const float *bins, int n_bins,
                          const float *table, int M, int D, void *out, int64_t *idx_out, fs2_stream_t stream);

/*
 * VariancePredictor, column-split form (model/modules.py:197-250; VarianceAdaptor.forward
 * :110-126). The two Conv1d(k=3) of G predictors that read the same input run as fs2_conv1d
 * launches whose workgroups each own a slice of the output columns (a small-M LayerNorm GEMM
 * would make every workgroup stream a whole weight matrix); the two LayerNorms move into these
 * row kernels. Every group is C = 256 columns (filter_size); one half-wave per (row, group).
 *
 * fs2_vp_norm: h = LayerNorm(y[m, g*C : (g+1)*C]; gamma[g], beta[g], eps) written as the bf16x3
 *   input planes of the second conv: out[m, g*2C + c] = bf16(h), out[m, g*2C + C + c] =
 *   bf16(h - bf16(h)).  (layer_norm_1 + dropout_1 (eval: identity), modules.py:218-222)
 * fs2_vp_head: per (row m = b*T + t, group g):
 *   p = (t >= lens[b]) ? 0 : dot(LayerNorm(y[m, g*C:(g+1)*C]; gamma2[g], beta2[g]), lin_w[g]) + lin_b[g]
 *   pred[g*B*T + m] = p                        (layer_norm_2, linear_layer, masked_fill :233-250)
 *   and for g == embed_group (>= 0) the pitch/energy embedding of fs2_variance_embed, in the
 *   same pass: v = target ? target[m] : (pred *= control); x[m, :D] += table[bucketize(v, bins)].
 */
int fs2_vp_norm(const float *y, int64_t y_row_stride, int M, int G, int C, const float *gamma, const float *beta,
                float eps, void *out, int64_t out_row_stride, fs2_stream_t stream);
int fs2_vp_head(const float *y, int64_t y_row_stride, int B, int T, int G, int C, const float *gamma,
                const float *beta, float eps, const float *lin_w, const float *lin_b, const int64_t *lens,
                float *pred, int embed_group, void *x, int x_dtype, int64_t x_row_stride, int D,
                const float *target, float control, const float *bins, int n_bins, const float *table,
                fs2_stream_t stream);

/*
 * fs2_vp_fused — G (1 or 2) whole VariancePredictors on the same bf16 input in ONE launch
 * (model/modules.py:197-250; VarianceAdaptor.forward :110-126), split-precision bf16x3 like the
 * column-split form above (w = w_hi + w_lo; conv1 x.w_hi + x.w_lo, h = h_hi + h_lo as bf16 planes,
 * conv2 h_hi.w_hi + h_hi.w_lo + h_lo.w_hi; f32 accumulation, LayerNorm, dot):
 *   h = LN1(relu(conv1_k3(x) + b1)); y = LN2(relu(conv2_k3(h) + b2))      (padding = 1 per utterance)
 *   pred[g*B*L + m] = (t >= lens[b]) ? 0 : dot(y[m], lin_w[g]) + lin_b[g]  (m = b*L + t)
 *   g == embed_group: v = target ? target[m] : (pred *= control);
 *                     x_out[m, :256] = bf16(x[m, :256] + table[bucketize(v, bins)])   (x_out != x)
 * Replaces conv1 + fs2_vp_norm + conv2 + fs2_vp_head (4 launches, 4 HBM intermediates) per set.
 * Channels 256 (filter_size = d_model), kernel 3. w: fs2_vp_fused_weight_elems(G) bf16 elements,
 * per predictor [4 quads][2 convs][24 k-steps][2 parts (hi, lo)][4][4][16][8]: element (q, c, s,
 * e, b, h, r, i) = part_e(W_c)[64q + 16b + r][32s + 8h + i] with W_c[n][tap*256 + ch] =
 * conv_c.weight[n][ch][tap]. vec: f32 [G][7][256] = conv1 bias, LN1 gamma, LN1 beta, conv2 bias,
 * LN2 gamma, LN2 beta, linear weight.
 */
typedef struct fs2_vp_fused_desc {
  const void *x;            /* bf16 [B*L, >= 256]                                                  */
  int64_t x_row_stride;
  const void *w;            /* bf16, fragment order (see above)                                    */
  const float *vec;         /* f32 [G][7][256]                                                     */
  const float *lin_b;       /* f32 [G]                                                             */
  float ln_eps;
  int B, L, G;
  const int64_t *lens;      /* [B] phoneme lengths (masked_fill)                                   */
  float *pred;              /* f32 [G, B*L]                                                        */
  int embed_group;          /* -1: none                                                            */
  void *x_out;              /* bf16 [B*L, >= 256]                                                  */
  int64_t x_out_row_stride;
  const float *target;      /* f32 [B*L] or NULL                                                   */
  float control;
  const float *bins;        /* f32 [n_bins - 1]                                                    */
  int n_bins;
  const float *table;       /* f32 [n_bins, 256]                                                   */
} fs2_vp_fused_desc;

int fs2_vp_fused(const fs2_vp_fused_desc *d, fs2_stream_t stream);
int64_t fs2_vp_fused_weight_elems(int G);

/*
 * LengthRegulator (model/modules.py:161-194 + utils/tools.py:360-378), split in two launches
 * so a caller without max_mel_len can read max(mel_len) in between (one D2H read per batch,
 * where the reference does B*L_max .item() syncs).
 *
 * fs2_lr_durations: per sequence, frames_i = max(trunc(d_i), 0) over ALL L positions,
 *   cum[b,i] = sum_{j<=i} frames_j (int32, saturating), mel_len[b] = sum (int64, not cropped).
 *   dur_kind FS2_DUR_I64: d int64 targets; FS2_DUR_F32: f32 durations (truncated like int());
 *   FS2_DUR_LOGPRED: d = f32 log-duration predictions, rounded like modules.py:132-135:
 *   d_rounded = clamp(round_half_even(exp(d) - 1) * d_control, min=0), written to d_rounded.
 * fs2_lr_expand: out[b,t,:] = (t < min(mel_len[b], T_out) ? x[b, src(b,t), :] : 0) (+ pe[t,:]),
 *   src(b,t) = first i with cum[b,i] > t.  pe (f32 [>=T_out, D]) may be NULL; a non-NULL pe
 *   fuses the Decoder's position_enc add (transformer/Models.py:158-160).  index_map (int32
 *   [B, T_out], -1 on padding) is optional; with index_map given, out may be NULL (only the
 *   map is written: the training gather's index-map-only call).  D must be a multiple of 8.
 *   out_cu (int32 [B+1], fs2_seq_layout) != NULL: packed output — only frames
 *   t < out_cu[b+1] - out_cu[b] are written, at row out_cu[b] + t.
 */
enum fs2_dur_kind { FS2_DUR_I64 = 0, FS2_DUR_F32 = 1, FS2_DUR_LOGPRED = 2 };

int fs2_lr_durations(const void *dur, int dur_kind, float d_control, int B, int L, int32_t *cum, int64_t *mel_len,
                     float *d_rounded, fs2_stream_t stream);
int fs2_lr_expand(const void *x, int x_dtype, const int32_t *cum, const int64_t *mel_len, int B, int L, int D,
                  int T_out, const float *pe, void *out, int out_dtype, int32_t *index_map, const int32_t *out_cu,
                  fs2_stream_t stream);

/*
 * fs2_lr_fused — the LengthRegulator + pad (model/modules.py:161-194, utils/tools.py:360-378) AND
 * the decoder's packed layout (fs2_seq_layout of layout_lens over T_out) in ONE launch, the
 * frames written packed: out[cu[b] + t, :] = x[b, src(b,t), :] (+ pe[t, :]) for t < clamp(
 * layout_lens[b], 0, T_out) (zeros for t >= mel_len[b]); cu / row_pos / rowmap as fs2_seq_layout.
 * Durations either scanned here (dur != NULL, dur_kind / d_control as fs2_lr_durations; cum,
 * mel_len and, for FS2_DUR_LOGPRED, d_rounded are written) or taken from an earlier
 * fs2_lr_durations (dur == NULL: cum_in, mel_len_in; the free-running path, whose host read of
 * max(mel_len) sits between the two). L <= 2048, B <= 4096, D % 8 == 0.
 */
int fs2_lr_fused(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control, const int32_t *cum_in,
                 const int64_t *mel_len_in, int B, int L, int D, int T_out, const float *pe,
                 const int64_t *layout_lens, int32_t *cu, int32_t *row_pos, int32_t *rowmap, void *out,
                 int out_dtype, int32_t *cum, int64_t *mel_len, float *d_rounded, fs2_stream_t stream);

/*
 * fs2_lr_fused_proj — fs2_lr_fused plus the decoder's first Q|K|V projection of the gathered frames
 * by linearity (SubLayers.py:39-41 on the LengthRegulator output, Models.py:145-152's PE added):
 * (x[b, src] + pe[t]) W^T + b = (x W^T)[b, src] + (pe W^T + b)[t], so
 * proj_out[cu[b] + t, :NP] = bf16(proj_src[b * L + src(b,t), :] + proj_pe[t, :]) (proj_src row
 * omitted for t >= mel_len[b]). proj_src: f32 [B * L, NP], the phoneme rows' projection (one
 * fs2_conv1d over B*L rows instead of the frames); proj_pe: f32 [>= T_out, NP] = pe W^T + b, a
 * per-weight table. NP % 8 == 0, NP <= 1536. With proj_out == NULL this is fs2_lr_fused.
 */
int fs2_lr_fused_proj(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control,
                      const int32_t *cum_in, const int64_t *mel_len_in, int B, int L, int D, int T_out,
                      const float *pe, const int64_t *layout_lens, int32_t *cu, int32_t *row_pos, int32_t *rowmap,
                      void *out, int out_dtype, int32_t *cum, int64_t *mel_len, float *d_rounded,
                      const float *proj_src, const float *proj_pe, int NP, void *proj_out, fs2_stream_t stream);

/* The reference's LengthRegulator.forward + pad (model/modules.py:161-194, utils/tools.py:360-378)
 * with a caller-known T_out (the teacher-forced / max_mel_len path) in ONE launch: duration scan
 * (cum, mel_len, d_rounded as fs2_lr_durations), gather (+ PE) into the padded [B, T_out, D] out,
 * zeros past min(mel_len, T_out), optional int32 [B, T_out] source map (-1 past the length). out
 * may be NULL with index_map given (map only; two launches then, as for L > 2048 phonemes). */
int fs2_length_regulate(const void *x, int x_dtype, const void *dur, int dur_kind, float d_control, int B, int L,
                        int D, int T_out, const float *pe, void *out, int out_dtype, int32_t *cum, int64_t *mel_len,
                        float *d_rounded, int32_t *index_map, fs2_stream_t stream);

/*
 * fs2_length_masks — get_mask_from_lengths (utils/tools.py:152-160): mask[b, t] = (t >= lens[b]),
 * bool [B, width], True = padding. The forward returns src_masks / mel_masks built this way.
 */
int fs2_length_masks(const int64_t *lens, int B, int width, bool *mask, fs2_stream_t stream);

/*
 * fs2_seq_layout — packed-sequence layout of B sequences of clamp(lens[b], 0, T) frames:
 *   cu[b] = sum_{j<b} len_j (int32 [B+1], cu[B] = total rows),
 *   row_pos[2r], row_pos[2r+1] = {frame, len} of packed row r (int32 [B*T][2], optional),
 *   rowmap[b*T + t] = t < len_b ? cu[b] + t : -1 (int32 [B*T], optional).
 * Two launches, no host sync. The Decoder's mel_masks lengths define its packing.
 */
int fs2_seq_layout(const int64_t *lens, int B, int T, int32_t *cu, int32_t *row_pos, int32_t *rowmap,
                   fs2_stream_t stream);

/*
 * fs2_hifigan_mrf — one HiFi-GAN V1 upsampling stage's multi-receptive-field block in ONE launch
 * (hifigan/models.py:20-45 ResBlock1 with kernels (3, 7, 11) x dilations (1, 3, 5), summed and
 * averaged, :152-158), for C = 32 or 64 channels (the last two stages):
 *   xs = sum_k ResBlock_k(x);  out = leaky_relu(xs / 3, out_slope)
 *   ResBlock_k: for d in (1, 3, 5): x = conv2(lrelu(conv1_d(lrelu(x, 0.1)) + b1, 0.1)) + b2 + x
 * x: the upsampler output bf16 [B, T, C]; x_act = lrelu(x, 0.1) (its second output); out bf16
 * [B, T, C] (must not alias either). Per-utterance zero padding at [0, T) for every conv.
 * w: fs2_hifigan_mrf_weight_elems(C) bf16, conv (chain j, pair p, second s) at element offset
 * sum_{j' < j} 6 k_{j'} C^2 + (2p + s) k_j C^2, each [k C/32 k-steps][C/16 blocks][4 h][16 r][8 e],
 * element (s, b, h, r, e) = W[16b + r][32s + 8h + e], W[n][tap C + c] = conv.weight[n][c][tap]
 * (weight norm folded); bias f32 [18][C] in the same conv order.
 */
int fs2_hifigan_mrf(const void *x, const void *x_act, const void *w, const float *bias, int B, int T, int C,
                    float out_slope, void *out, fs2_stream_t stream);
int64_t fs2_hifigan_mrf_weight_elems(int C);

/*
 * fs2_hifigan_pair — one ResBlock1 dilation pair at C = 128 or 64 (the second / third upsampling
 * stage, hifigan/models.py:34-45) in ONE launch:
 *   y = conv2(lrelu(conv1_d(lrelu(x, 0.1)) + b1, 0.1)) + b2 + x (+ xs)
 *   out = y (out_act = 0) or lrelu(y * out_scale, out_slope) (out_act = 1: the stage's last pair,
 *   out_scale = 1 / num_kernels)
 * x bf16 [B, T, C] (must not alias out); xs optional bf16 [B, T, C] (the running
 * multi-receptive-field sum; may alias out); ks in {3, 7, 11}, dilation 1..5 (conv1; conv2 has
 * dilation 1); w1 / w2 each ks * C * C bf16 in the fs2_hifigan_mrf per-conv layout
 * [ks * C/32 k-steps][C/16 blocks][4 h][16 r][8 e]; b1 / b2 f32 [C]. Per-utterance zero padding at
 * [0, T) for both convs. Replaces the pair's two fs2_conv1d launches and their t / lrelu(x)
 * round trips through HBM.
 */
int fs2_hifigan_pair(const void *x, const void *w1, const float *b1, const void *w2, const float *b2, int B, int T,
                     int C, int ks, int dilation, const void *xs, float out_scale, float out_slope, int out_act,
                     void *out, fs2_stream_t stream);

/*
 * fs2_hifigan_post — the generator's conv_post + tanh (hifigan/models.py:145, 159-162):
 *   out[b, t] = tanh(bias + sum_{k<ks, c<C} w[k][c] x[b, t + k - ks/2, c])
 * x bf16 [B, T, C] (the leaky_relu'd last-stage output), out f32 [B, T] (the waveform), w bf16
 * [ks][C] (tap-major: the reference's conv_post.weight[0].T), per-utterance zero padding. C = 32,
 * ks = 7, T even. A streaming one-channel kernel (replaces an MFMA conv with N padded to 4).
 */
int fs2_hifigan_post(const void *x, const void *w, float bias, int B, int T, int C, int ks, void *out,
                     fs2_stream_t stream);

/*
 * Training-step kernels (train.py step; training.py's FFTBlockFn / Conv1dFn backward):
 * fs2_res_ln_fwd — y = masked_fill(LayerNorm(dropout(a, p_drop) + res), t >= lens[b], 0) over
 *   R = B*T rows of D = 256 (transformer/SubLayers.py:54-57,90-93, Layers.py:27-30): a f32, res
 *   f32 or bf16, y f32 (+ optional bf16 copy y_bf), saved xhat f32 [R, D] and rstd f32 [R]. Dropout
 *   keep bits are a counter hash of (*seed, salt, row, column) (seed: one device int64, may be
 *   advanced between steps inside a captured graph); p_drop = 0 -> no dropout (seed unused).
 * fs2_res_ln_bwd — its backward: dres = dLN (f32 [R, D]), da = dres * keep / (1 - p) (bf16 [R, D]),
 *   dgamma, dbeta f32 [D] and dbias f32 [D] (optional: sum over rows of da = the producing conv's
 *   bias gradient); accumulate != 0 adds into them. Deterministic (fixed-order partial sums in ws).
 * fs2_colsum — out[n] (+)= sum over R rows of x[r, n] (f32 or bf16), deterministic.
 * fs2_conv_wgrad — Conv1d weight gradient without an unfolded copy:
 *   dw[n][c][k] (+)= sum_{b,t} dy[b,t,n] x[b, t+k-pad, c] (x zero outside [0, T) per sequence),
 *   db[n] (+)= sum dy[b,t,n] (optional); dy f32 or bf16 [B*T, N], x bf16 [B*T, C], KS in
 *   {1, 3, 5, 9}, N and C multiples of 8. MFMA bf16, f32 accumulation, deterministic.
 *   split_rows > 0: rows [i*split_rows, (i+1)*split_rows) of dw / db go to (dw, dw1, dw2)[i] /
 *   (db, db1, db2)[i] (2 or 3 parts: the separate Q, K, V parameters of one fused projection).
 *   defer != 0: only the partials are written to ws ([S][KS][N][C] for dW, then [S][N] for db;
 *   S = fs2_conv_wgrad_splits(...)), for fs2_reduce_batch_launch; dw / db unused.
 */
int fs2_res_ln_fwd(const float *a, const void *res, int res_dtype, const float *gamma, const float *beta,
                   const int64_t *lens, int64_t R, int T, int D, float eps, float p_drop, const int64_t *seed,
                   int salt, float *y, void *y_bf, float *xhat, float *rstd, fs2_stream_t stream);
int64_t fs2_res_ln_bwd_ws_bytes(int D);
int fs2_res_ln_bwd(const float *dy, const float *xhat, const float *rstd, const float *gamma, const int64_t *lens,
                   int64_t R, int T, int D, float p_drop, const int64_t *seed, int salt, float *dres, void *da,
                   float *dgamma, float *dbeta, float *dbias, int accumulate, int defer, float *ws,
                   int64_t ws_bytes, fs2_stream_t stream);
/* fs2_relu_ln_fwd / fs2_relu_ln_bwd — one VariancePredictor layer after its conv in train mode,
 *   y = dropout(LayerNorm(relu(a)))  (model/modules.py:218-235; R rows of D = 256), y f32 (+ optional
 *   bf16 copy), saved xhat / rstd; the backward takes a again (relu mask) and gives da bf16 and
 *   dgamma / dbeta / dbias (the conv's bias gradient, optional), accumulate as fs2_res_ln_bwd.
 *   ws: fs2_res_ln_bwd_ws_bytes(D). */
int fs2_relu_ln_fwd(const float *a, const float *gamma, const float *beta, int64_t R, int D, float eps, float p_drop,
                    const int64_t *seed, int salt, float *y, void *y_bf, float *xhat, float *rstd,
                    fs2_stream_t stream);
int fs2_relu_ln_bwd(const float *dy, const float *a, const float *xhat, const float *rstd, const float *gamma,
                    int64_t R, int D, float p_drop, const int64_t *seed, int salt, void *da, float *dgamma,
                    float *dbeta, float *dbias, int accumulate, int defer, float *ws, int64_t ws_bytes,
                    fs2_stream_t stream);
/* fs2_relu_ln_head_fwd / fs2_relu_ln_head_bwd — the VariancePredictor's second layer WITH its head
 *   (model/modules.py:230-250, train mode): fs2_relu_ln_fwd's relu + LayerNorm + dropout and
 *   hout[r] = hmask[r] ? 0 : y[r] . hw + hb[0] (linear_layer + squeeze + masked_fill) in one launch; y
 *   itself is not written (optional bf16 copy). The backward takes dout (the predictor output's
 *   gradient) in place of dy (dy[r][c] = masked ? 0 : dout[r] * hw[c]) and also gives the head's
 *   dhw [D] / dhb [1]; defer != 0: the LN partials (first fs2_res_ln_bwd_ws_bytes(D) bytes of ws, S =
 *   fs2_ln_bwd_parts(R)) and the head's [S][D + 4] partials after them go to fs2_reduce_batch_launch
 *   (kinds 0 and 2). ws: fs2_relu_ln_head_bwd_ws_bytes(D). Replaces the reference's F.linear +
 *   masked_fill pair (and their backward) for the bf16 training path. */
int fs2_relu_ln_head_fwd(const float *a, const float *gamma, const float *beta, int64_t R, int D, float eps,
                         float p_drop, const int64_t *seed, int salt, void *y_bf, float *xhat, float *rstd,
                         const float *hw, const float *hb, const bool *hmask, float *hout, fs2_stream_t stream);
int64_t fs2_relu_ln_head_bwd_ws_bytes(int D);
int fs2_relu_ln_head_bwd(const float *dout, const bool *hmask, const float *hw, const float *beta, const float *a,
                         const float *xhat, const float *rstd, const float *gamma, int64_t R, int D, float p_drop,
                         const int64_t *seed, int salt, void *da, float *dgamma, float *dbeta, float *dbias,
                         float *dhw, float *dhb, int accumulate, int defer, float *ws, int64_t ws_bytes,
                         fs2_stream_t stream);
/* fs2_embedding_bwd — nn.Embedding's weight gradient (transformer/Models.py:82 src_word_emb with
 *   padding_idx, model/modules.py:80-100 pitch / energy tables, fastspeech2.py:101-110 speaker /
 *   emotion tables): out[v][:] (+)= sum over i with tokens[i] == v, in increasing i, of dy[i][:]
 *   (deterministic, no atomics); row padding_idx (< 0: none) untouched unless accumulate == 0 (then
 *   zero). D <= 256. */
int fs2_embedding_bwd(const int64_t *tokens, int64_t n, const float *dy, int64_t dy_row_stride, int V, int D,
                      int padding_idx, float *out, int accumulate, fs2_stream_t stream);
int64_t fs2_colsum_ws_bytes(int N);
int fs2_colsum(const void *x, int dtype, int64_t R, int N, int64_t row_stride, float *out, int accumulate, float *ws,
               int64_t ws_bytes, fs2_stream_t stream);
int64_t fs2_conv_wgrad_ws_bytes(int B, int T, int N, int C, int KS);
int fs2_conv_wgrad(const void *dy, int dy_dtype, int64_t dy_row_stride, const void *x, int64_t x_row_stride, int B,
                   int T, int N, int C, int KS, int pad, float *dw, float *db, int accumulate, int split_rows,
                   float *dw1, float *dw2, float *db1, float *db2, int defer, float *ws, int64_t ws_bytes,
                   fs2_stream_t stream);

/*
 * fs2_pack_train_plan / fs2_pack_train — every MFMA weight image of a training step in one launch.
 * Per descriptor (a host array completed by fs2_pack_train_plan, then copied to device memory
 * for fs2_pack_train):
 *   f32_copy = 0: src f32 [N][C][KS] -> fwd bf16 [N_tot][KS][C] rows n_off.. (optional) and
 *                 tr bf16 [C][KS][N_tot] columns n_off.. with tr[c][k][n] = src[n][c][KS-1-k]
 *                 (the input-gradient conv's weight; optional);
 *   f32_copy = 1: src f32 [N] -> ((float *)fwd)[n_off + n] (a fused projection's bias).
 * fs2_pack_train_plan fills tiles_c / blk0 and *blocks (the fs2_pack_train grid size).
 */
typedef struct fs2_pack_desc {
  const float *src;
  void *fwd;
  void *tr;
  int N, C, KS, n_off, N_tot, f32_copy;
  int C_tot;         /* row length of the forward image (>= C: channel padding left as is); 0 = C */
  int tiles_c, blk0; /* filled by fs2_pack_train_plan */
} fs2_pack_desc;
int fs2_pack_train_plan(fs2_pack_desc *descs, int nd, int *blocks);
int fs2_pack_train(const fs2_pack_desc *descs_dev, int nd, int blocks, fs2_stream_t stream);

/*
 * FastSpeech2Loss (model/loss.py:5-92) on device, no host sync:
 * fs2_loss_fwd — out[0..5] = (total, mel L1, postnet L1, pitch MSE, energy MSE, log-duration MSE)
 *   over the masks, stats[0..3] = the element counts (kept for the backward); ws: fs2_loss_ws_bytes().
 *   mel / postnet f32 [B, T, n_mel] contiguous, mel_tgt f32 rows at b*tgt_bs + t*tgt_ts (the target
 *   cropped to T frames), masks bool (1 = valid), log_d target = log(d_tgt + 1). Deterministic.
 * fs2_loss_bwd — d(prediction) for all five from the upstream gradients grad_out[6] of out[0..5]
 *   and the forward's stats (sign(err) for the L1 terms, 0 at err == 0, as torch's abs backward).
 */
typedef struct fs2_loss_args {
  const float *mel, *postnet, *mel_tgt;
  int64_t tgt_bs, tgt_ts;
  const unsigned char *mel_valid;
  int B, T, n_mel;
  const float *p_pred, *p_tgt;
  const unsigned char *p_mask;
  int64_t n_p;
  const float *e_pred, *e_tgt;
  const unsigned char *e_mask;
  int64_t n_e;
  const float *logd_pred;
  const int64_t *d_tgt;
  const unsigned char *d_mask;
  int64_t n_d;
} fs2_loss_args;
int64_t fs2_loss_ws_bytes(void);
int fs2_loss_fwd(const fs2_loss_args *a, float *out, float *stats, float *ws, int64_t ws_bytes, fs2_stream_t stream);
int fs2_loss_bwd(const fs2_loss_args *a, const float *grad_out, const float *stats, float *d_mel, float *d_postnet,
                 float *d_pitch, float *d_energy, float *d_logd, fs2_stream_t stream);

/*
 * PostNet layer in train mode (transformer/Layers.py:92-137 with BatchNorm1d on batch statistics):
 * fs2_bn_train_fwd — z f32 [R, C] (the conv output, R = B*T frames, C % 4 == 0, C <= 1024):
 *   mean / var over the R rows (biased; deterministic Chan combination of per-block two-pass
 *   moments), running_mean / running_var updated with momentum (unbiased variance; both may be
 *   null), y = dropout(act(gamma * (z - mean) * rstd + beta)) (+ residual) with act = tanh when
 *   use_tanh; y_bf (bf16) and / or y_f32 written; mean / rstd [C] saved.
 * fs2_bn_train_bwd — dz bf16 [R, C] from dy f32 (recomputing zhat, tanh and the dropout bits);
 *   dgamma / dbeta (+)=. ws: fs2_bn_train_ws_bytes(C) for both.
 */
int64_t fs2_bn_train_ws_bytes(int C);
int fs2_bn_train_fwd(const float *z, int64_t R, int C, const float *gamma, const float *beta, float eps,
                     float momentum, float *running_mean, float *running_var, int use_tanh, float p_drop,
                     const int64_t *seed, int salt, const float *residual, void *y_bf, float *y_f32, float *mean,
                     float *rstd, float *ws, int64_t ws_bytes, fs2_stream_t stream);
int fs2_bn_train_bwd(const float *dy, const float *z, int64_t R, int C, const float *gamma, const float *beta,
                     const float *mean, const float *rstd, int use_tanh, float p_drop, const int64_t *seed, int salt,
                     void *dz, float *dgamma, float *dbeta, int accumulate, float *ws, int64_t ws_bytes,
                     fs2_stream_t stream);

/*
 * fs2_adam_flat — nn.utils.clip_grad_norm_(max_norm) + torch.optim.Adam's step (fused / capturable
 * semantics: m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2, p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t)
 * + eps), L2 weight decay added to g) for parameters whose gradients are one flat f32 buffer
 * (train.py:92-95 through ScheduledOptim). params_dev: device array of np descriptors in flat order
 * (param, exp_avg, exp_avg_sq, step counter (f32, advanced by 1 here), offset and length in the
 * flat buffer). lr from lr_dev when non-null (a captured step reads the current Noam lr), else lr.
 * max_norm <= 0: no clipping; else the clipped gradients are written back. Deterministic norm.
 * ws: fs2_adam_ws_bytes().
 */
typedef struct fs2_adam_param {
  float *p, *m, *v, *step;
  int64_t off, numel;
} fs2_adam_param;
int64_t fs2_adam_ws_bytes(void);
int fs2_adam_flat(float *grads, int64_t n, const fs2_adam_param *params_dev, int np, const float *lr_dev, float lr,
                  float beta1, float beta2, float eps, float weight_decay, float max_norm, float *ws,
                  int64_t ws_bytes, fs2_stream_t stream);

/*
 * fs2_reduce_batch_launch — up to FS2_REDUCE_BATCH_MAX deferred split-partial reductions in one
 * launch (the fused training nodes' gradient finishes, batched after the backward): per descriptor
 * out[m] (+)= sum over s < S of part[s * M + m] (fixed order), scattered by kind:
 *   0: m -> (out0 | out1 | out2)[m / split][m % split] (LayerNorm gamma / beta / bias, Q|K|V biases);
 *   1: weight-gradient partials m = (k*N + n)*C + c -> out_{n / split}[((n % split)*C + c)*KS + k];
 *   2: m < split -> out0[m], m == split -> out1[0], m > split ignored (a vector + one scalar: the
 *      VariancePredictor head's weight and bias, fs2_relu_ln_head_bwd).
 * blk0 is filled in. Partials come from fs2_conv_wgrad / fs2_res_ln_bwd / fs2_relu_ln_bwd with
 * defer != 0 (fs2_conv_wgrad_splits / fs2_ln_bwd_parts give their S).
 */
#define FS2_REDUCE_BATCH_MAX 32
typedef struct fs2_reduce_desc {
  const float *part;
  int64_t M;
  int S, kind, KS, N, C, split, accumulate, pad_;
  float *out0, *out1, *out2;
  int64_t blk0;
} fs2_reduce_desc;
typedef struct fs2_reduce_batch {
  int n, pad_;
  fs2_reduce_desc d[FS2_REDUCE_BATCH_MAX];
} fs2_reduce_batch;
int fs2_reduce_batch_launch(fs2_reduce_batch *a, fs2_stream_t stream);
int fs2_conv_wgrad_splits(int B, int T, int N, int C, int KS);
int fs2_ln_bwd_parts(int64_t R);

/*
 * fs2_lr_backward — gradient of the LengthRegulator gather (training; model/modules.py:161-194 +
 *   the decoder crop transformer/Models.py:154-162): dx[b, i, :] = sum over t in
 *   [cum[b, i-1], cum[b, i]) with t < T of dy[b, t, :] (cum from fs2_lr_durations, int32 [B, L]; dy
 *   f32 [B, T, D], dx f32 [B, L, D], contiguous). Frames summed in order: deterministic, no atomics.
 */
int fs2_lr_backward(const float *dy, const int32_t *cum, int B, int L, int D, int T, float *dx, fs2_stream_t stream);

/* Library identification. fs2_build_id: sha256 (hex, first 16 digits) of the sources the library
 * was compiled from (the .hip and .h files of csrc and include/fs2hip.h, in name order), embedded by the build
 * (__graft_entry__.build_hip); fs2amd._lib.load() refuses a library whose id differs from the
 * sources beside it. */
const char *fs2_version(void);
const char *fs2_build_id(void);
const char *fs2_status_string(int status);

/*
 * The PostNet's valid-region form for mostly-padding batches (free-running synthesis; the
 * reference computes the PostNet, transformer/Layers.py:92-137, on every padded frame):
 * fs2_pack_rows — padded rows -> packed rows: row i of a (and of b, optional) goes to row
 *   rowmap[i] (>= 0; fs2_seq_layout's rowmap) of packed_a (packed_b); rows of a_row_bytes /
 *   b_row_bytes bytes (multiples of 16).
 * fs2_postnet_assemble — packed PostNet output back to [B, T, C] f32: out[b, t] = y_packed[rowmap[b*T+t]]
 *   where the packed rows are exact (with len2 = cu[b+1] - cu[b] of the layout (fs2_seq_layout_margin):
 *   t < len2 - reach, or every t when len2 == T), else the
 *   row t - (T - reach) of tail [reach, C] for the last reach frames, else const_row [C] (the
 *   PostNet of all-padding input). C % 4 == 0.
 */
int fs2_pack_rows(const void *a, int a_row_bytes, void *packed_a, const void *b, int b_row_bytes, void *packed_b,
                  const int32_t *rowmap, int64_t n_rows, fs2_stream_t stream);
int fs2_postnet_assemble(const float *y_packed, const int32_t *rowmap, const int32_t *cu, int B, int T, int C,
                         const float *const_row, const float *tail, int reach, float *out, fs2_stream_t stream);

/*
 * fs2_seq_layout_margin — fs2_seq_layout over transformed lengths: len'[b] = T when
 *   lens[b] + 2*margin > T, else lens[b] + margin (the PostNet valid-region rows: each utterance's
 *   frames + margin frames of its padding), clamped to [0, T]; margin 0 = fs2_seq_layout. B <= 4096.
 * fs2_len_stats — meta[0..2] = {max(lens), sum(lens), *bad_counter (0 if NULL)} as int32 (lengths
 *   clamped at 0 and saturated at 2^31 - 1): the free-running path's one device->host read
 *   (synthesize_chinese_pinyin.py:140-145 sizes the decoder from max(mel_len)) in one launch.
 */
int fs2_seq_layout_margin(const int64_t *lens, int B, int T, int margin, int32_t *cu, int32_t *row_pos,
                          int32_t *rowmap, fs2_stream_t stream);
int fs2_len_stats(const int64_t *lens, int B, const int32_t *bad_counter, int32_t *meta, fs2_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* FS2HIP_H */
