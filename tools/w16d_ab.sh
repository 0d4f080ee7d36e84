#!/bin/bash
# 16 waves (2 x 8 of 64 x 32) on the decoder LN ring tiles (FS2_LN_W16DEC=1): parity tests with it on, probes, bench A/B
D=gpurun_out/w16d; mkdir -p $D
FS2_LN_W16DEC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_model.py tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
for i in 1 2; do
  for V in 0 1; do
    for K in fc conv1; do
      FS2_LN_W16DEC=$V timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 50 > $D/p.txt 2>&1 || exit $?
      echo "W16D=$V $(tail -n 1 $D/p.txt)" >> $D/summary.txt
    done
  done
done
bash tools/ab_multi.sh w16dab "FS2_LN_W16DEC=0" "FS2_LN_W16DEC=1"
