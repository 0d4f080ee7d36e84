#!/bin/bash
# Attention A/B: the attention tests first (correctness of the default kernel), then standalone
# HIP-event timing of the decoder-shape kernel in both forms (FS2_ATTN32=1: 32 queries per wave on
# 32x32x16 MFMAs; 0: 16 queries per wave), then one forward trace. Every GPU step has its own time
# limit; the chain stops at the first failure.
TAG=${1:-attn}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_train.py tests/test_gpu_graphs.py -k "attention or attn or graph" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  FS2_ATTN32=$v timeout -k 10 120 python tools/kernel_probe.py attn --time >> $O/attn_time.log 2>&1 || { tail -5 $O/attn_time.log; exit 1; }
  echo "attn32=$v $(tail -1 $O/attn_time.log)"
done
bash tools/fwd_trace.sh $TAG || exit 1
