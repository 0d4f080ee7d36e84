#!/bin/bash
# SynthGraphs stage 2 as two graphs (first decoder block, then the rest): graph tests, probes
# (split / FS2_SYNTH_SPLIT=0 / eager), free-running trace
O=gpurun_out/r5s1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_graphs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
FS2_SYNTH_SPLIT=0 timeout -k 10 200 python tools/free_probe.py > $O/free_onegraph.log 2>&1 || { tail -20 $O/free_onegraph.log; exit 1; }
grep -v amdgpu.ids $O/free_onegraph.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
bash tools/free_trace.sh r5s1/free || exit 1
