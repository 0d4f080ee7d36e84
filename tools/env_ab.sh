#!/bin/bash
# A/B of an environment switch on the headline bench (alternated runs on one box), then one
# rocprofv3 forward trace with the switch at its default.
# usage: tools/env_ab.sh NAME VALUE_A VALUE_B [TAG]
N=$1; A=$2; B=$3; O=gpurun_out/${4:-envab}; mkdir -p $O
for V in $A $B $A $B; do
  env $N=$V timeout -k 10 300 python bench.py --extra 0 --vocoder 0 --cpu-baseline 0 --steps 30 > $O/b_$V.log 2>&1 || { tail -20 $O/b_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$V.log').read().strip().splitlines()[-1]); print('$N=$V', d['ms_per_step'])"
done
if [ -z "$NOTRACE" ]; then bash tools/fwd_trace.sh ${4:-envab}_trace; fi
