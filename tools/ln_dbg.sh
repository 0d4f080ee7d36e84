#!/bin/bash
# where the LN-epilogue ring kernels spend their time: FS2_CONV_DEBUG bit 0 skips the K loop,
# bit 1 the epilogue (analysis only; outputs are garbage)
D=gpurun_out/lndbg; mkdir -p $D
for K in fc conv1 qkv conv9; do
  for V in 0 1 2 3; do
    FS2_CONV_DEBUG=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "DEBUG=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
