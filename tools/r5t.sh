#!/bin/bash
# round-5 t: fused PostNet tail, software-pipelined fragment reads
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
for K in wconv pn_tail pn_tail_fused; do
  timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 20 > $O/$K.log 2>&1 || { tail -20 $O/$K.log; exit 1; }
  echo "$(tail -1 $O/$K.log)"
done
