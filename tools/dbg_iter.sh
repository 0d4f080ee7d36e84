#!/bin/bash
mkdir -p gpurun_out/dbg2
for D in 0 2 4 8 16 28 3; do
  for K in conv1; do
    FS2_CONV_DEBUG=$D timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 40 2>/dev/null | sed "s/^/DBG=$D /" >> gpurun_out/dbg2/summary.txt || exit $?
  done
done
