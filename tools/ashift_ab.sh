#!/bin/bash
D=gpurun_out/ashift; mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for V in 0 1 0 1; do
  for K in conv9 enc_conv9; do
    FS2_CONV_ASHIFT=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
    echo "ASHIFT=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
  done
done
FS2_CONV_ASHIFT=0 timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576 --reps 30 > $D/s0.txt 2>&1 || exit $?
FS2_CONV_ASHIFT=1 timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576 --reps 30 > $D/s1.txt 2>&1 || exit $?
bash tools/ab_multi.sh ashiftab "FS2_CONV_ASHIFT=0" "FS2_CONV_ASHIFT=1"
