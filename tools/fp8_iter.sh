#!/bin/bash
mkdir -p gpurun_out/fp8c
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/fp8c/t.log 2>&1
rc=$?; echo "fp8 tests rc=$rc" >> gpurun_out/fp8c/summary.txt; [ $rc -gt 1 ] && exit $rc
for D in fp8 bf16; do
  timeout -k 10 400 python bench.py --dtype $D --cpu-baseline 0 > gpurun_out/fp8c/bench_$D.log 2>&1 || exit $?
  echo "$D $(tail -1 gpurun_out/fp8c/bench_$D.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["roofline"]["kernel_ms"], j["roofline"]["achieved"], j["roofline"]["frac"])')" >> gpurun_out/fp8c/summary.txt
done
