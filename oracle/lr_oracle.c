/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * Plain-C restatement of the reference LengthRegulator, the integer/index part of the hot path:
 *   model/modules.py:182-190  expand(): for each phoneme i, repeat row i max(int(d_i), 0) times
 *                                       (int() truncates toward zero; .item() per phoneme)
 *   model/modules.py:167-180  LR():     concatenate per sequence, mel_len = uncropped length,
 *                                       pad() to max_len when given, else to max(mel_len)
 *   utils/tools.py:360-378    pad():    F.pad with (0, max_len - len): zero-fill or crop;
 *                                       `if mel_max_length:` -> a max_len of 0 means "not given"
 * Pinned by tests/test_lr_oracle_c.py against tests/golden/lr_cases.npz and the per-case
 * index maps, which tests/golden/gen_golden.py captured from the reference itself.
 *
 * dur_kind 0: int64 durations; 1: float32 durations.
 */
#include <stdint.h>
#include <string.h>

static int64_t frames_i64(const int64_t *d, int64_t i) { return d[i] > 0 ? d[i] : 0; }
static int64_t frames_f32(const float *d, int64_t i) {
  float v = d[i];
  if (!(v > 0.0f)) return 0;
  return (int64_t)v; /* C truncation == Python int() for finite values */
}

/* mel_len[b] for every sequence; returns max(mel_len) (the output length when max_len is not given). */
int64_t lr_oracle_lengths(const void *dur, int dur_kind, int B, int L, int64_t *mel_len) {
  int64_t mx = 0;
  for (int b = 0; b < B; ++b) {
    int64_t s = 0;
    for (int i = 0; i < L; ++i) {
      int64_t k = (int64_t)b * L + i;
      s += dur_kind == 0 ? frames_i64((const int64_t *)dur, k) : frames_f32((const float *)dur, k);
    }
    mel_len[b] = s;
    if (s > mx) mx = s;
  }
  return mx;
}

/* index_map[b, t] = source phoneme of output frame t, -1 on padding; T_out columns. */
void lr_oracle_index_map(const void *dur, int dur_kind, int B, int L, int T_out, int32_t *index_map) {
  for (int b = 0; b < B; ++b) {
    int64_t t = 0;
    for (int i = 0; i < L && t < T_out; ++i) {
      int64_t k = (int64_t)b * L + i;
      int64_t n = dur_kind == 0 ? frames_i64((const int64_t *)dur, k) : frames_f32((const float *)dur, k);
      for (int64_t r = 0; r < n && t < T_out; ++r) index_map[(int64_t)b * T_out + t++] = i;
    }
    for (; t < T_out; ++t) index_map[(int64_t)b * T_out + t] = -1;
  }
}

/* out[b, t, :] = x[b, src, :] or 0 — float32 rows of D elements. */
void lr_oracle_expand_f32(const float *x, const void *dur, int dur_kind, int B, int L, int D, int T_out,
                          float *out, int32_t *index_map) {
  lr_oracle_index_map(dur, dur_kind, B, L, T_out, index_map);
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < T_out; ++t) {
      int32_t s = index_map[(int64_t)b * T_out + t];
      float *o = out + ((int64_t)b * T_out + t) * D;
      if (s < 0)
        memset(o, 0, sizeof(float) * (size_t)D);
      else
        memcpy(o, x + ((int64_t)b * L + s) * D, sizeof(float) * (size_t)D);
    }
}
