#!/bin/bash
# round-5 z: phase stamps inside fs2_enc_attn_block (trace build), tests, A/B, trace
O=gpurun_out/r5z; mkdir -p $O
FS2_LIB=$PWD/abl/libfs2hip_enctrace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/enc_trace.py > $O/enc_trace.log 2>&1 || { tail -20 $O/enc_trace.log; exit 1; }
grep -v amdgpu.ids $O/enc_trace.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_enc_block.py tests/test_gpu_model.py tests/test_gpu_graphs.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 0 1; do
  FS2_ENC_HALF=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "ENC_HALF=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
bash tools/fwd_trace.sh r5z/trace_run || exit 1
head -10 $O/trace_run/forward_kernels.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/train_tests.log 2>&1 || { tail -40 $O/train_tests.log; exit 1; }
tail -1 $O/train_tests.log
GRAPH=1 bash tools/prof_train.sh r5z/train || exit 1
python3 tools/train_steps.py $(ls $O/train/trace/*kernel_trace.csv | head -1) > $O/train_steps.txt 2>&1
head -8 $O/train_steps.txt
