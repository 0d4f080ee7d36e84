#!/bin/bash
# round-5 checkpoint g: graphs / model / fp8 / ffn tests, decoder FFN (PRE + Q|K|V) phase trace,
# free-running timing (eager and SynthGraphs), the bench line, forward and free-running traces.
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_model.py tests/test_gpu_fp8.py tests/test_gpu_ffn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --dec-pre > $O/dec_trace.log 2>&1 || { tail -20 $O/dec_trace.log; exit 1; }
grep -v amdgpu.ids $O/dec_trace.log
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --enc --no-qkv > $O/enc_trace.log 2>&1 || { tail -20 $O/enc_trace.log; exit 1; }
grep -v amdgpu.ids $O/enc_trace.log | tail -9
timeout -k 10 120 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 && tail -1 $O/free_eager.log
timeout -k 10 120 python tools/free_probe.py > $O/free_graphs.log 2>&1 && tail -1 $O/free_graphs.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5g/trace_run || exit 1
bash tools/free_trace.sh r5g/free || exit 1
