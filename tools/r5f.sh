#!/bin/bash
# round-5 checkpoint f: HIP graph event-node probe, FFN tests, encoder FFN phase traces (PRE form,
# without the Q|K|V epilogue), the bench line, the graphed training line, forward + free-running
# traces. Each GPU step has its own time limit; stop at the first failure.
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 120 python tools/event_probe.py > $O/event_probe.log 2>&1; grep -v amdgpu.ids $O/event_probe.log | tail -8
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_graphs.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
FS2_LIB=$PWD/abl/libfs2hip_trace.so FS2_LIB_ALLOW_MISSING=1 timeout -k 10 120 python tools/ffn_trace.py --enc --no-qkv > $O/enc_trace.log 2>&1 || { tail -20 $O/enc_trace.log; exit 1; }
grep -v amdgpu.ids $O/enc_trace.log
for V in "" "FS2_LR_STORE=plain" "FS2_LR_STORE=sc1" "FS2_FFN_PRE_ENC=0" "FS2_QKV_FUSED=2" "FS2_ATTN32_FORM=8x2"; do
  env $V timeout -k 10 120 python tools/fwd_breakdown.py --tag "${V:-default}" >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  tail -1 $O/ab.log | cut -c1-600
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --mode train --graph 1 --steps 20 --warmup 5 > $O/train_graph.log 2>&1 || { tail -20 $O/train_graph.log; exit 1; }
tail -1 $O/train_graph.log | cut -c1-300
bash tools/fwd_trace.sh r5f/trace_run || exit 1
bash tools/free_trace.sh r5f/free || exit 1
