#!/bin/bash
D=gpurun_out/deepb; mkdir -p $D
FS2_CONV_DEEPB=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -x -q --timeout 200 --timeout-method thread -k "conv" > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for V in 0 1 2; do
    for K in enc_conv9 conv9; do
      FS2_CONV_DEEPB=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
      echo "DEEPB=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
bash tools/ab_multi.sh deepbab "FS2_CONV_DEEPB=0" "FS2_CONV_DEEPB=1" "FS2_CONV_DEEPB=2"
