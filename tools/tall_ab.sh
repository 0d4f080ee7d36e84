#!/bin/bash
# tall 256x128 deep-ring conv kernel: parity under FS2_CONV_TALL=1, then sweep + bench A/B
D=gpurun_out/tall; mkdir -p $D
FS2_CONV_TALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > $D/t.log 2>&1 || exit $?
for V in "FS2_CONV_TALL=0" "FS2_CONV_TALL=1" "FS2_CONV_TALL=1 FS2_CONV_SPLITK=0"; do
  env $V timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576,24883,25600,27520,32768 --reps 30 > $D/s.txt 2>&1 || exit $?
  echo "$V $(grep M= $D/s.txt | awk '{print $2, $3}' | tr '\n' ' ')" >> $D/summary.txt
done
bash tools/ab_multi.sh tallab "FS2_CONV_TALL=0" "FS2_CONV_TALL=1"
