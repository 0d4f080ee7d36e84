#!/bin/bash
# 8-wave 128x128 conv tiles (FS2_CONV_W8=1): GPU suite with it on, probes, bench A/B
D=gpurun_out/cw8; mkdir -p $D
FS2_CONV_W8=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for V in 0 1; do
    for K in conv9 qkv postnet_last; do
      FS2_CONV_W8=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
      echo "CW8=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
bash tools/ab_multi.sh cw8ab "FS2_CONV_W8=0" "FS2_CONV_W8=1"
