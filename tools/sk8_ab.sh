#!/bin/bash
# phased stream-K: parity, then sweep + bench A/B vs the whole-rounds + remainder split
D=gpurun_out/sk8; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "splitk or conv1d_bias" > $D/t.log 2>&1 || exit $?
for V in "FS2_CONV_8PSK=0" "FS2_CONV_8PSK=1"; do
  env $V timeout -k 10 200 python tools/m_sweep.py --ms 16384,24576,24883,25600,27520,32768,40000 --reps 30 > $D/s.txt 2>&1 || exit $?
  echo "$V $(grep M= $D/s.txt | awk '{print $2, $3}' | tr '\n' ' ')" >> $D/summary.txt
done
bash tools/ab_multi.sh sk8ab "FS2_CONV_8PSK=0" "FS2_CONV_8PSK=1"
