#!/bin/bash
# VariancePredictor sets on 64-row tiles (FS2_VP_TILE=64) vs 32: the VP / model tests under 64,
# probe timing (cold, after a 512 MB flush) and forward traces. Each GPU step has its own limit.
TAG=${1:-r4q}
O=gpurun_out/$TAG; mkdir -p $O
FS2_VP_TILE=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "vp or variance or predictor or model or forward" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests64.log 2>&1 || { tail -20 $O/tests64.log; exit 1; }
tail -1 $O/tests64.log
for rep in 1 2; do for t in 32 64; do for k in vpf_dp vpf_en; do
  FS2_VP_TILE=$t timeout -k 10 120 python tools/kernel_probe.py $k --time --reps 10 --flush 512 >> $O/vp_time.log 2>&1 || { tail -5 $O/vp_time.log; exit 1; }
  echo "tile=$t $(tail -1 $O/vp_time.log)"
done; done; done
FS2_VP_TILE=64 bash tools/fwd_trace.sh $TAG/t64 || exit 1
bash tools/fwd_trace.sh $TAG/t32 || exit 1
for t in t32 t64; do echo "$t: $(grep -E 'vp_fused' $O/$t/forward_kernels.txt | awk '{printf "%s ", $(NF-2)}') $(tail -1 $O/$t/forward_kernels.txt)"; done
