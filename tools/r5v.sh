#!/bin/bash
# round-5 v: the encoder attention sub-layer in one launch (fs2_enc_attn_block)
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_enc_block.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/enc.log 2>&1 || { tail -40 $O/enc.log; exit 1; }
tail -3 $O/enc.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_graphs.py tests/test_gpu_fp8.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_ENC_BLOCK=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "ENC_BLOCK=$V $(tail -1 $O/ab$V.log | cut -c1-450)"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5v/trace_run || exit 1
head -22 $O/trace_run/forward_kernels.txt
for V in 0 1; do
  FS2_FFN_PRE_64=$V timeout -k 10 200 python tools/free_probe.py > $O/free$V.log 2>&1 || { tail -20 $O/free$V.log; exit 1; }
  echo "FFN_PRE_64=$V $(grep -v amdgpu.ids $O/free$V.log | tail -1)"
done
bash tools/free_trace.sh r5v/free || exit 1
