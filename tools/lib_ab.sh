#!/bin/bash
# A/B of two library builds (FS2_LIB) on the decoder probes and the headline bench.
# usage: tools/lib_ab.sh <old.so>
OLD=$1
for L in new old new old; do
  if [ $L = old ]; then export FS2_LIB=$OLD FS2_LIB_ALLOW_MISSING=1; else unset FS2_LIB FS2_LIB_ALLOW_MISSING; fi
  for K in ${PROBES:-fc conv1 qkv conv9 attn}; do
    timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 | sed "s/^/$L /" || exit 1
  done
  timeout -k 10 300 python bench.py --extra 0 --cpu-baseline 0 --steps 20 | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L bench', d['value'], d['ms_per_step'])" || exit 1
done
