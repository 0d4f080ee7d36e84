#!/bin/bash
mkdir -p gpurun_out/tr3
timeout -k 10 600 python -m pytest tests/test_gpu_train.py -q -p no:cacheprovider > gpurun_out/tr3/t.log 2>&1
rc=$?; echo "train tests rc=$rc" >> gpurun_out/tr3/summary.txt; [ $rc -gt 1 ] && exit $rc
for D in bf16 fp32; do
  timeout -k 10 400 python bench.py --mode train --dtype $D --steps 10 --warmup 3 > gpurun_out/tr3/bench_$D.log 2>&1 || exit $?
  echo "train $D $(tail -1 gpurun_out/tr3/bench_$D.log | cut -c100-200)" >> gpurun_out/tr3/summary.txt
done
