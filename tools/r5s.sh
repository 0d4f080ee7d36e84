#!/bin/bash
# round-5 s: the fused PostNet tail launch alone (graph-timed) against wconv and the N = 80 tail,
# with ablation builds (abl/libfs2hip_tail1.so: no tail MFMA loop; tail2: no tail at all)
O=gpurun_out/r5s; mkdir -p $O
for K in wconv pn_tail pn_tail_fused; do
  timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 20 > $O/$K.log 2>&1 || { tail -20 $O/$K.log; exit 1; }
  echo "$(tail -1 $O/$K.log)"
done
for A in 1 2; do
  FS2_LIB=$PWD/abl/libfs2hip_tail$A.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/kernel_probe.py pn_tail_fused --time --reps 20 > $O/abl$A.log 2>&1 || { tail -20 $O/abl$A.log; exit 1; }
  echo "ablate $A: $(tail -1 $O/abl$A.log)"
done
