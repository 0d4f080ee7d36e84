#!/bin/bash
# bf16 mel copy for PostNet's first conv: tests, probe A/B, bench A/B on one box
D=gpurun_out/melbf; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for K in postnet_first postnet_first_bf; do
    timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "$(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
bash tools/ab_multi.sh melbfab "FS2_MEL_BF16=0" "FS2_MEL_BF16=1"
