#!/bin/bash
# round-5 checkpoint: GPU suite, smoke, the default bench line, forward trace, PMC passes over eager
# forwards (-> the PRE kernel's traffic record), graphed training line, free-running probe + trace
O=gpurun_out/r5ck; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash tools/fwd_trace.sh r5ck/trace_run || exit 1
bash tools/pmc_fwd.sh r5ck > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pre_traffic.py gpurun_out/pmcf_r5ck/table.json profiles/r5ck/pmc_forward.json $O/ffn_pre_traffic.json
timeout -k 10 400 python bench.py --mode train --graph 1 > $O/train.log 2>&1 || { tail -30 $O/train.log; exit 1; }
grep -h '"metric"' $O/train.log | cut -c1-260
timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
grep -v amdgpu.ids $O/free.log | tail -1
timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
grep -v amdgpu.ids $O/free_eager.log | tail -1
bash tools/free_trace.sh r5ck/free || exit 1
