#!/bin/bash
# round-5 y: encoder attention block, head-split form (FS2_ENC_HALF A/B)
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_enc_block.py tests/test_gpu_model.py tests/test_gpu_graphs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_ENC_HALF=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "ENC_HALF=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
bash tools/fwd_trace.sh r5y/trace_run || exit 1
head -10 $O/trace_run/forward_kernels.txt
