#!/bin/bash
# round-5 k: LengthRegulator projection as column-owning row batches; decoder FFN PRE sub-phase trace
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lr_fused" > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --dec-pre > $O/dec_trace.log 2>&1 || { tail -20 $O/dec_trace.log; exit 1; }
grep -v amdgpu.ids $O/dec_trace.log
for V in 1 0; do
  FS2_LR_PROJ=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "LR_PROJ=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
bash tools/fwd_trace.sh r5k/trace_run || exit 1
