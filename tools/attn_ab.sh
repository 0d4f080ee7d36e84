#!/bin/bash
# attention variants: parity tests under each, then per-launch time at the cfg2 decoder shape
D=gpurun_out/attn_ab; mkdir -p $D
for V in 1 0 2 3; do
  FS2_ATTN_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $D/t$V.log 2>&1 || exit $?
  FS2_ATTN_VARIANT=$V timeout -k 10 120 python tools/kernel_probe.py attn --time --reps 50 > $D/p$V.txt 2>&1 || exit $?
  echo "variant $V: $(tail -1 $D/t$V.log) | $(tail -1 $D/p$V.txt)" >> $D/summary.txt
done
