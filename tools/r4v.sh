#!/bin/bash
# cond_kernel with the weight loads issued before the id gathers: conditioning tests, the probe
# timing, and a forward trace.
TAG=${1:-r4v}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "cond or speaker or emotion or forward" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/kernel_probe.py cond --time > $O/cond.log 2>&1 || { tail -5 $O/cond.log; exit 1; }
tail -1 $O/cond.log
bash tools/fwd_trace.sh $TAG/trace_run || exit 1
grep cond_kernel $O/trace_run/forward_kernels.txt
