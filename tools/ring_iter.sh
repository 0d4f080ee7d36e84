#!/bin/bash
mkdir -p gpurun_out/ring1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/ring1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ring1/summary.txt; [ $rc -gt 1 ] && exit $rc
for R in 1 0; do
  FS2_CONV_RING=$R timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/ring1/bench_r$R.log 2>&1 || exit $?
  echo "ring=$R $(tail -1 gpurun_out/ring1/bench_r$R.log | cut -c1-160)" >> gpurun_out/ring1/summary.txt
done
for K in enc_ln vp conv1; do
  FS2_CONV_RING=1 timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 20 >> gpurun_out/ring1/summary.txt 2>&1 || exit $?
  FS2_CONV_RING=0 timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 20 >> gpurun_out/ring1/summary.txt 2>&1 || exit $?
done
