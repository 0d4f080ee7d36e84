#!/bin/bash
# round-5 w: fs2_enc_attn_block with a pipelined weight ring
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_enc_block.py tests/test_gpu_model.py tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_ENC_BLOCK=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "ENC_BLOCK=$V $(tail -1 $O/ab$V.log | cut -c1-450)"
done
bash tools/fwd_trace.sh r5w/trace_run || exit 1
head -12 $O/trace_run/forward_kernels.txt
