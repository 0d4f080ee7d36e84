#!/bin/bash
mkdir -p gpurun_out/grp1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -q -p no:cacheprovider -x > gpurun_out/grp1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/grp1/summary.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/m_sweep.py --ms 24883,27520,32768 >> gpurun_out/grp1/summary.txt 2>&1 || exit $?
timeout -k 10 120 python tools/kernel_probe.py conv9 --time --reps 20 >> gpurun_out/grp1/summary.txt 2>&1 || exit $?
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d gpurun_out/grp1/pmc_conv9_$C -o pmc --output-format csv -- python3 tools/kernel_probe.py conv9 --reps 10 > gpurun_out/grp1/pmc_$C.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --cpu-baseline 0 > gpurun_out/grp1/bench.log 2>&1 || exit $?
tail -1 gpurun_out/grp1/bench.log | cut -c1-200 >> gpurun_out/grp1/summary.txt
