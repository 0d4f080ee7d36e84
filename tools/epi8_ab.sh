#!/bin/bash
D=gpurun_out/epi8; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
for V in 0 1 0 1; do
  for K in qkv conv9 postnet; do
    FS2_LN_PAIRS=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "WIDE=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
bash tools/ab_multi.sh epi8ab "FS2_LN_PAIRS=0" "FS2_LN_PAIRS=1"
