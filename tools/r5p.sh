#!/bin/bash
# round-5 p: LengthRegulator launch alone, graph-replayed (kernel_probe --time): no projection,
# projection variants (FS2_LR_PROJ_DBG: 8 wave-3 x gather; 1/2/4 no table / phoneme loads / stores)
O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 120 python tools/kernel_probe.py lr_fused --time --reps 20 > $O/lr.log 2>&1 || { tail -20 $O/lr.log; exit 1; }
echo "lr_fused: $(tail -1 $O/lr.log)"
for V in 0 8 1 2 4 7 15; do
  FS2_LR_PROJ_DBG=$V timeout -k 10 120 python tools/kernel_probe.py lr_proj --time --reps 20 > $O/p$V.log 2>&1 || { tail -20 $O/p$V.log; exit 1; }
  echo "lr_proj DBG=$V: $(tail -1 $O/p$V.log)"
done
