#!/bin/bash
# Encoder FFN forms at the cfg2 encoder shape (4096 rows): fused (cost-model default, 64x2, 112x4)
# against the two-launch form (conv k9 + ReLU, then conv k1 + residual + LN). HIP events, graphs.
TAG=${1:-r4n}
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
for a in "enc_ffn" "enc_ffn --nsplit 2 --tile-rows 64" "enc_ffn --nsplit 4 --tile-rows 112" "enc_conv9" "enc_ln"; do
  timeout -k 10 120 python tools/kernel_probe.py $a --time >> $O/enc.log 2>&1 || { tail -5 $O/enc.log; exit 1; }
  echo "$a: $(tail -1 $O/enc.log)"
done
done
