#!/bin/bash
# GPU tests, then the bench at 1 / 2 / 4 utterance-group streams.
mkdir -p gpurun_out/st1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/st1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/st1/summary.txt; [ $rc -gt 1 ] && exit $rc
for S in 1 2 4; do
  FS2_STREAMS=$S timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/st1/bench_s$S.log 2>&1 || exit $?
  echo "streams=$S $(tail -1 gpurun_out/st1/bench_s$S.log | cut -c1-200)" >> gpurun_out/st1/summary.txt
done
