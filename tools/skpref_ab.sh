#!/bin/bash
# full GPU suite (defaults), then small-M split-K A/B: probes + bench
D=gpurun_out/skpref; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
for V in 0 1; do
  for K in vp enc_conv9 enc_ln; do
    FS2_CONV_SKPREF=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "SKPREF=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
bash tools/ab_multi.sh skprefab "FS2_CONV_SKPREF=0" "FS2_CONV_SKPREF=1"
