#!/bin/bash
# round-5 final checkpoint: GPU suite, smoke, bench line, forward trace, free-running probes
# (graphed / eager / FS2_FFN_PRE64=0) + traces, vocoder profile
O=gpurun_out/r5fin; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --extra 0 > $O/bench_driver.log 2>&1 || { tail -30 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
FS2_FFN_PRE64=0 timeout -k 10 200 python tools/free_probe.py > $O/free_nopre.log 2>&1 || { tail -20 $O/free_nopre.log; exit 1; }
grep -v amdgpu.ids $O/free_nopre.log | tail -1
bash tools/free_trace.sh r5fin/free || exit 1
bash tools/fwd_trace.sh r5fin/trace_run || exit 1
