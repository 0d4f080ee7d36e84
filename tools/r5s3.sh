#!/bin/bash
# numpy views on the pinned meta vector (host poll / checks), split stage 2 off by default:
# graph + model tests, free-running probes, free trace
O=gpurun_out/r5s3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
bash tools/free_trace.sh r5s3/free || exit 1
