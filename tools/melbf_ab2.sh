#!/bin/bash
D=gpurun_out/melbf2; mkdir -p $D
for i in 1 2; do
  for V in 1 0; do
    FS2_CONV_PHASED=$V timeout -k 10 120 python tools/kernel_probe.py postnet_first_bf --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "PHASED=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
bash tools/ab_multi.sh melbfab2 "FS2_MEL_BF16=0" "FS2_MEL_BF16=1" "FS2_MEL_BF16=0" "FS2_MEL_BF16=1"
