#!/bin/bash
# Attention A/B: standalone HIP-event timing of the decoder-shape kernel, one forward trace, and
# the attention tests. Every GPU step has its own time limit; the chain stops at the first failure.
TAG=${1:-attn}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 python tools/kernel_probe.py attn --time > gpurun_out/$TAG/attn_time.log 2>&1 || { tail -5 gpurun_out/$TAG/attn_time.log; exit 1; }
tail -1 gpurun_out/$TAG/attn_time.log
bash tools/fwd_trace.sh $TAG || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_graphs.py -k "attention or attn or graph" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 || { tail -20 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
