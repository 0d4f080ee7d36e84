#!/bin/bash
# Same-box bench A/B over several env settings, alternated twice.  usage: ab_multi.sh tag "ENV=.. ENV2=.." "..." ...
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
for i in 1 2; do
  j=0
  for V in "$@"; do
    j=$((j+1))
    env $V timeout -k 10 300 python bench.py --cpu-baseline 0 > $D/bench_${j}_$i.log 2>&1 || exit $?
    echo "[$V] run$i $(tail -1 $D/bench_${j}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')" >> $D/summary.txt
  done
done
