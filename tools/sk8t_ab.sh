#!/bin/bash
# 8p kernel without the stream-K bookkeeping (no spills): parity tests, then same-box lib A/B
D=gpurun_out/sk8t; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
PROBES="conv9 postnet postnet_first_bf" bash tools/ab_lib.sh oldlib/libfs2hip_prev.so sk8tab
