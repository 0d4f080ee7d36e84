#!/bin/bash
# A/B of the ring kernel's L2 weight prefetch (FS2_L2PF) on the small-M LayerNorm GEMM probes, then the bench.
for P in ${KLIST:-}; do
  for K in vp enc_ln; do
    FS2_L2PF=$P timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 | sed "s/^/l2pf=$P /" || exit 1
  done
done
for P in ${PLIST:-1 2 1 2}; do
  FS2_L2PF=$P timeout -k 10 300 python bench.py --extra 0 --cpu-baseline 0 --steps 20 | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('l2pf=$P bench', d['value'], d['ms_per_step'])" || exit 1
done
