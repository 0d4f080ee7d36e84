#!/bin/bash
# Attention + vocoder A/B: attention standalone timing, the vocoder / attention / graph tests, a
# vocoder profile and a forward trace. Each GPU step has its own time limit; stop at the first failure.
TAG=${1:-ab}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 python tools/kernel_probe.py attn --time > $O/attn_time.log 2>&1 || { tail -5 $O/attn_time.log; exit 1; }
tail -1 $O/attn_time.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoder.py tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_graphs.py -k "vocoder or mrf or generator or attention or attn or graph" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_train_kernels.py -k adam -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_adam.log 2>&1 || { tail -20 $O/tests_adam.log; exit 1; }
tail -1 $O/tests_adam.log
bash tools/prof_voc.sh $TAG && bash tools/fwd_trace.sh $TAG
