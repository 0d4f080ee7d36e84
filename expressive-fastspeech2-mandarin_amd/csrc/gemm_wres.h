// Weight-resident projection GEMM (gemm_wres.hip), dispatched from fs2_conv1d (conv_gemm.hip).
#pragma once
#include "fs2_common.h"

struct WresArgs {
  const void *x;          // bf16 rows of >= K elements
  int64_t xs;             // x row stride (elements)
  const void *w;          // packed bf16 [N][K] (Conv1d k=1 / Linear)
  const float *bias;      // [N] or NULL
  void *out;              // bf16 (or f32 with out_f32) [rows][os]
  int64_t os;
  int M;                  // rows (padded layout) ...
  const int32_t *rows_dev;  // ... or the device-side active row count (packed layout), or NULL
  int N, K;               // N % 128 == 0, K in {64, 128, 192, 256}
  int relu;               // 0: y = acc + bias, 1: relu(acc + bias)
  int out_f32;            // f32 output (16-byte stores) instead of bf16
  uint32_t x_bytes, w_bytes;
  int out_sc1;            // set by wres_launch: write-through bf16 stores (conv_common.h env_out_sc1)
};

// true when the launch was taken (shape / dtype covered); the caller falls back otherwise
bool wres_launch(const WresArgs &a, int num_cus, hipStream_t s);
