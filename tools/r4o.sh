#!/bin/bash
# PostNet tail on 8 waves (FS2_PN_TAIL8=1): the wconv / PostNet tests under it, then two forward
# traces (4-wave default and 8-wave tail). Each GPU step has its own time limit.
TAG=${1:-r4o}
O=gpurun_out/$TAG; mkdir -p $O
FS2_PN_TAIL8=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_tail8.log 2>&1 || { tail -20 $O/tests_tail8.log; exit 1; }
tail -1 $O/tests_tail8.log
FS2_PN_TAIL8=1 bash tools/fwd_trace.sh $TAG/tail8 || exit 1
bash tools/fwd_trace.sh $TAG/tail4 || exit 1
grep pn_tail $O/tail8/forward_kernels.txt $O/tail4/forward_kernels.txt
