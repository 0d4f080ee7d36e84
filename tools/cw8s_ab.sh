#!/bin/bash
# 8-wave 64- and 32-row conv tiles (FS2_CONV_W8S=1): GPU suite with it on, probes, bench A/B
D=gpurun_out/cw8s; mkdir -p $D
FS2_CONV_W8S=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for V in 0 1; do
    for K in enc_conv9; do
      FS2_CONV_W8S=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
      echo "CW8S=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
bash tools/ab_multi.sh cw8sab "FS2_CONV_W8S=0" "FS2_CONV_W8S=1"
