#!/bin/bash
# round-5 checkpoint, second half: the conditioning fold A/B (FS2_ENC_COND), graphed training line,
# free-running probe + trace
O=gpurun_out/r5ck2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_enc_block.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/enc_tests.log 2>&1 || { tail -40 $O/enc_tests.log; exit 1; }
tail -1 $O/enc_tests.log
bash tools/fwd_trace.sh r5ck2/trace_nocond || exit 1
FS2_ENC_COND=1 bash tools/fwd_trace.sh r5ck2/trace_cond || exit 1
timeout -k 10 400 python bench.py --mode train --graph 1 > $O/train.log 2>&1 || { tail -30 $O/train.log; exit 1; }
grep -h '"metric"' $O/train.log | cut -c1-260
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
bash tools/free_trace.sh r5ck2/free || exit 1
