#!/bin/bash
# round-5 r: fused PostNet tail, 4 compute waves x 2 row blocks (LDS-bandwidth form)
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_PN_TAIL_FUSED=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "PN_TAIL_FUSED=$V $(tail -1 $O/ab$V.log | cut -c1-300)"
done
bash tools/fwd_trace.sh r5r/trace_run || exit 1
tail -6 $O/trace_run/forward_kernels.txt
