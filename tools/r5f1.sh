#!/bin/bash
# free-running: fc + LN prologue on the packed 64-row FFN tiles (FS2_FFN_PRE64), the embed-fold
# first encoder block in SynthGraphs' stage 1; tests, then probes (graphed / eager, PRE64 on / off)
O=gpurun_out/r5f1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_graphs.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
FS2_FFN_PRE64=0 timeout -k 10 200 python tools/free_probe.py > $O/free_nopre.log 2>&1 || { tail -20 $O/free_nopre.log; exit 1; }
grep -v amdgpu.ids $O/free_nopre.log | tail -1
bash tools/free_trace.sh r5f1/free || exit 1
bash tools/free_trace.sh r5f1/free_eager --eager || exit 1
