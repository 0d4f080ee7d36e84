#!/bin/bash
mkdir -p gpurun_out/rb1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/rb1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/rb1/summary.txt; [ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  for X in 1 0; do
    for K in conv1; do
      FS2_CONV_RB=$X timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 2>/dev/null | sed "s/^/RB=$X run$i /" >> gpurun_out/rb1/summary.txt || exit $?
    done
    FS2_CONV_RB=$X timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/rb1/bench_${X}_$i.log 2>&1 || exit $?
    echo "RB=$X run$i bench $(tail -1 gpurun_out/rb1/bench_${X}_$i.log | cut -c80-120)" >> gpurun_out/rb1/summary.txt
  done
done
