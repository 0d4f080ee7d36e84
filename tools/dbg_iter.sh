#!/bin/bash
mkdir -p gpurun_out/dbg1
for D in 0 1 2 3; do
  for K in conv1 enc_ln; do
    FS2_CONV_DEBUG=$D timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 2>/dev/null | sed "s/^/DBG=$D /" >> gpurun_out/dbg1/summary.txt || exit $?
  done
done
