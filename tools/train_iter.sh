#!/bin/bash
mkdir -p gpurun_out/tr1
timeout -k 10 600 python -m pytest tests/test_gpu_train.py -q -p no:cacheprovider > gpurun_out/tr1/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc" >> gpurun_out/tr1/summary.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/tr1/tests.log 2>&1
rc=$?; echo "all gpu tests rc=$rc" >> gpurun_out/tr1/summary.txt; [ $rc -gt 1 ] && exit $rc
for D in bf16 fp32; do
  timeout -k 10 400 python bench.py --mode train --dtype $D --steps 10 --warmup 3 > gpurun_out/tr1/bench_train_$D.log 2>&1 || exit $?
  echo "train $D $(tail -1 gpurun_out/tr1/bench_train_$D.log)" >> gpurun_out/tr1/summary.txt
done
