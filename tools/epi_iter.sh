#!/bin/bash
mkdir -p gpurun_out/epi1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/epi1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/epi1/summary.txt; [ $rc -gt 1 ] && exit $rc
for K in conv1 enc_ln vp qkv conv9 postnet; do
  timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 >> gpurun_out/epi1/summary.txt 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/epi1/bench_$i.log 2>&1 || exit $?
  echo "bench $(tail -1 gpurun_out/epi1/bench_$i.log | cut -c80-150)" >> gpurun_out/epi1/summary.txt
done
