#!/bin/bash
D=gpurun_out/narrow; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for V in 0 1 0 1; do
  for K in postnet_last postnet_first; do
    FS2_CONV_NARROW=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "NARROW=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
bash tools/ab_multi.sh narrowab "FS2_CONV_NARROW=0" "FS2_CONV_NARROW=1"
