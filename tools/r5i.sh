#!/bin/bash
# round-5 A/B i: utterance groups on parallel streams (FS2_STREAMS) under graph replay, the headline
# bench only (50 timed steps after 20), alternated to separate box drift from the variant.
O=gpurun_out/r5i; mkdir -p $O
for V in "FS2_STREAMS=1" "FS2_STREAMS=2" "FS2_STREAMS=4" "FS2_STREAMS=1" "FS2_STREAMS=2"; do
  env $V timeout -k 10 200 python bench.py --steps 50 --warmup 20 --extra 0 --cpu-baseline 0 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$V $(tail -1 $O/b.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
FS2_STREAMS=2 bash tools/fwd_trace.sh r5i/trace_s2 || exit 1
