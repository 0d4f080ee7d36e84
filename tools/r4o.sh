#!/bin/bash
# PostNet weight-stream L2 warm-up (FS2_PN_PREFETCH, default on) and the 8-wave tail
# (FS2_PN_TAIL8=1): the wconv / PostNet / packed tests, then forward traces for each form. Each GPU
# step has its own time limit; stop at the first failure.
TAG=${1:-r4o}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py tests/test_gpu_model.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
FS2_PN_TAIL8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_wconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_tail8.log 2>&1 || { tail -20 $O/tests_tail8.log; exit 1; }
tail -1 $O/tests_tail8.log
bash tools/fwd_trace.sh $TAG/pf || exit 1
FS2_PN_PREFETCH=0 bash tools/fwd_trace.sh $TAG/nopf || exit 1
FS2_PN_TAIL8=1 bash tools/fwd_trace.sh $TAG/pf_tail8 || exit 1
for t in pf nopf pf_tail8; do echo "$t: $(grep -E 'pn_head|wconv|pn_tail' $O/$t/forward_kernels.txt | awk '{printf "%s ", $(NF-2)}')"; done
