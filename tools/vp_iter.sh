#!/bin/bash
mkdir -p gpurun_out/vp1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -p no:cacheprovider -k "split_precision or vp or ln" > gpurun_out/vp1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/vp1/summary.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/flip_rate.py >> gpurun_out/vp1/summary.txt 2>&1 || exit $?
for V in bf16x3 fp32; do
  FS2_HIP_VP_DTYPE=$V timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/vp1/bench_$V.log 2>&1 || exit $?
  echo "vp=$V $(tail -1 gpurun_out/vp1/bench_$V.log | cut -c80-150)" >> gpurun_out/vp1/summary.txt
done
