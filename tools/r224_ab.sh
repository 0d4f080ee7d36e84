#!/bin/bash
# 224-row phased tiles for one-round launches (PostNet k=5): parity tests, probes, bench A/B
D=gpurun_out/r224; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for V in 0 1; do
    for K in postnet postnet_first_bf; do
      FS2_CONV_8P224=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
      echo "8P224=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
bash tools/ab_multi.sh r224ab "FS2_CONV_8P224=0" "FS2_CONV_8P224=1"
