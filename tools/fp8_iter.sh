#!/bin/bash
mkdir -p gpurun_out/fp8b
timeout -k 10 600 python -m pytest tests/test_gpu_fp8.py -q -s -p no:cacheprovider > gpurun_out/fp8b/t.log 2>&1
rc=$?; echo "fp8 tests rc=$rc" >> gpurun_out/fp8b/summary.txt; [ $rc -gt 1 ] && exit $rc
for D in fp8 bf16; do
  timeout -k 10 400 python bench.py --dtype $D --cpu-baseline 0 > gpurun_out/fp8b/bench_$D.log 2>&1 || exit $?
  echo "$D $(tail -1 gpurun_out/fp8b/bench_$D.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["roofline"]["kernel_ms"], j["roofline"]["achieved"], j["roofline"]["frac"])')" >> gpurun_out/fp8b/summary.txt
done
