#!/bin/bash
# round-5 checkpoint e: focused GPU tests (graphs, model, fp8, ops, packed, train), the encoder
# FFN phase trace (abl/libfs2hip_trace.so, -DFFN_TRACE=1), attention probe timing, then the bench
# line and the free-running trace (tools/checkpoint.sh without the full suite / PMC).
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_graphs.py tests/test_gpu_model.py tests/test_gpu_fp8.py tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_train.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -2 $O/first.log
timeout -k 10 120 python tools/kernel_probe.py attn --time > $O/attn_time.log 2>&1 || { tail -20 $O/attn_time.log; exit 1; }
tail -1 $O/attn_time.log
for R in 32 64 128; do
  for K in lr_fused lr_fused4; do
    FS2_LR_ROWS=$R timeout -k 10 120 python tools/kernel_probe.py $K --time >> $O/lr_rows.log 2>&1 || { tail -20 $O/lr_rows.log; exit 1; }
    echo "rows=$R $(tail -1 $O/lr_rows.log)"
  done
done
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --enc > $O/enc_trace.log 2>&1 || { tail -20 $O/enc_trace.log; exit 1; }
grep -v amdgpu.ids $O/enc_trace.log
SKIP_TESTS=1 SKIP_TRACE=1 SKIP_PMC=1 bash tools/checkpoint.sh r5e
