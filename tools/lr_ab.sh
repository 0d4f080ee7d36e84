#!/bin/bash
D=gpurun_out/lrab; mkdir -p $D
for V in 1 2 3; do
  FS2_LR_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -k "lr or length" > $D/t$V.log 2>&1 || exit $?
done
for i in 1 2; do
  for V in 0 1 2 3; do
    for K in lr lr4; do
      FS2_LR_VARIANT=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 100 > $D/p.txt 2>&1 || exit $?
      echo "LR_VARIANT=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
