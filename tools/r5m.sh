#!/bin/bash
# round-5 m: FFN vectors by LDS-DMA (no load->store waits at kernel start)
# half of the tile DMA; LR projection v2. FFN / packed / model tests, trace, breakdown, bench.
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_packed.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --dec-pre > $O/dec_trace.log 2>&1 || { tail -20 $O/dec_trace.log; exit 1; }
grep -v amdgpu.ids $O/dec_trace.log
timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -1 $O/ab.log | cut -c1-420
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5m/trace_run || exit 1
