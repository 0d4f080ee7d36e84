#!/bin/bash
# attention kernel change: its GPU tests + the model goldens, graph-timed probe, bench
O=gpurun_out/${1:-attn}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/kernel_probe.py attn --time 2>&1 | tail -1 || exit 1
timeout -k 10 120 python tools/free_probe.py || exit 1
for V in 1 2; do
  timeout -k 10 300 python bench.py --extra 0 --vocoder 0 --cpu-baseline 0 --steps 30 > $O/bench_$V.log 2>&1 || { tail -20 $O/bench_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$V.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
done
