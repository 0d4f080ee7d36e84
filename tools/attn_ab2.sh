#!/bin/bash
D=gpurun_out/attn2; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $D/t_model.log 2>&1 || exit $?
for V in 4 5; do
  FS2_ATTN_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $D/t_attn$V.log 2>&1 || exit $?
done
for V in 2 4 5 0; do
  FS2_ATTN_VARIANT=$V timeout -k 10 120 python tools/kernel_probe.py attn --time --reps 50 > $D/p.txt 2>&1 || exit $?
  echo "attn variant $V: $(tail -n 1 $D/p.txt)" >> $D/summary.txt
done
bash tools/ab_multi.sh attn2ab "FS2_ATTN_VARIANT=2" "FS2_ATTN_VARIANT=4" "FS2_ATTN_VARIANT=5"
