#!/bin/bash
# deep rings with raw barriers: parity (tall conv, attention variants), then sweeps + bench A/B
D=gpurun_out/r1e; mkdir -p $D
FS2_CONV_TALL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > $D/t_tall.log 2>&1 || exit $?
for V in 1 3; do
  FS2_ATTN_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $D/t_attn$V.log 2>&1 || exit $?
done
for V in 2 1 3 0; do
  FS2_ATTN_VARIANT=$V timeout -k 10 120 python tools/kernel_probe.py attn --time --reps 50 > $D/p.txt 2>&1 || exit $?
  echo "attn variant $V: $(tail -1 $D/p.txt)" >> $D/summary.txt
done
for V in "FS2_CONV_TALL=0" "FS2_CONV_TALL=1"; do
  env $V timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576,24883,25600,27520,32768 --reps 30 > $D/s.txt 2>&1 || exit $?
  echo "$V $(grep M= $D/s.txt | awk '{print $2, $3}' | tr '\n' ' ')" >> $D/summary.txt
done
