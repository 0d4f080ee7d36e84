#!/bin/bash
# round-5 x: the first encoder block builds its input and the masks (fs2_enc_embed_attn_block)
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_enc_block.py tests/test_gpu_model.py tests/test_gpu_graphs.py tests/test_gpu_packed.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_ENC_EMBED=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "ENC_EMBED=$V $(tail -1 $O/ab$V.log | cut -c1-200)"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5x/trace_run || exit 1
head -8 $O/trace_run/forward_kernels.txt
