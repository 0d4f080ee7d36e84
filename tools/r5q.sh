#!/bin/bash
# round-5 q: the PostNet's last two convs in one launch (wconv_kernel<5, 512, 1, true>)
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py tests/test_gpu_model.py tests/test_gpu_ffn.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
for V in 1 0; do
  FS2_PN_TAIL_FUSED=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "PN_TAIL_FUSED=$V $(tail -1 $O/ab$V.log | cut -c1-420)"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5q/trace_run || exit 1
