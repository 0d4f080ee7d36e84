#!/bin/bash
# round-5 j: the decoder's first Q|K|V by linearity in the LengthRegulator launch
# (fs2_lr_fused_proj): packed / model / graphs / pipeline tests, forward breakdown A/B
# (FS2_LR_PROJ), bench line, forward trace.
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_model.py tests/test_gpu_graphs.py tests/test_gpu_pipeline.py tests/test_gpu_fp8.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0 1; do
  FS2_LR_PROJ=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "LR_PROJ=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5j/trace_run || exit 1
