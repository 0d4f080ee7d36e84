#!/bin/bash
# A/B of the small-M LayerNorm tile (FS2_LN_SMALLM_ROWS) on the variance predictor and encoder LN probes.
for R in 16 32 64; do
  for K in vp enc_ln; do
    FS2_LN_SMALLM_ROWS=$R timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 | sed "s/^/rows=$R /" || exit 1
  done
done
