#!/bin/bash
# GPU tests, then an alternated A/B of one environment switch on the headline bench, then a
# forward trace at the default. usage: tools/ab_check.sh TAG NAME A B
O=gpurun_out/$1; N=$2; A=$3; B=$4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for V in $A $B $A $B; do
  env $N=$V timeout -k 10 300 python bench.py --extra 0 --vocoder 0 --cpu-baseline 0 --steps 30 > $O/b_$V.log 2>&1 || { tail -20 $O/b_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$V.log').read().strip().splitlines()[-1]); print('$N=$V', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline'].get('with_next_qkv'))"
done
timeout -k 10 120 python tools/free_probe.py || exit 1
bash tools/fwd_trace.sh $1_trace
