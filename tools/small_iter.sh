#!/bin/bash
# small-launch changes (fused seq layout, cond butterfly): tests, then a bench kernel trace
D=gpurun_out/small; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
bash tools/trace_bench.sh small_trace
