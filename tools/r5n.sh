#!/bin/bash
# round-5 n: LengthRegulator projection with 16-byte stores (A/B FS2_LR_PROJ)
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lr_fused" > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_LR_PROJ=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "LR_PROJ=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
bash tools/fwd_trace.sh r5n/trace_run || exit 1
grep -n "lr_fused\|gemm_wres" $O/trace_run/forward_kernels.txt
