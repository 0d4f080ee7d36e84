#!/bin/bash
# VP warm-up cap 24 (energy set fully covered): VP tests, cold probe timing, forward trace.
TAG=${1:-r4s}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "vp or variance or forward" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for k in vpf_dp vpf_en; do
  timeout -k 10 120 python tools/kernel_probe.py $k --time --reps 10 --flush 512 >> $O/vp_time.log 2>&1 || { tail -5 $O/vp_time.log; exit 1; }
  echo "$(tail -1 $O/vp_time.log)"
done; done
bash tools/fwd_trace.sh $TAG || exit 1
grep vp_fused $O/forward_kernels.txt
