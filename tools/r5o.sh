#!/bin/bash
# round-5 o: where the LengthRegulator projection's time goes (FS2_LR_PROJ_DBG: 1 no table loads,
# 2 no phoneme loads, 4 no stores; timing only)
O=gpurun_out/r5o; mkdir -p $O
for V in 0 1 2 3 4 7; do
  FS2_LR_PROJ_DBG=$V timeout -k 10 120 python tools/fwd_breakdown.py > $O/ab$V.log 2>&1 || { tail -20 $O/ab$V.log; exit 1; }
  echo "DBG=$V $(tail -1 $O/ab$V.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["us"]["va:lr"], r["us"].get("dec:qkv0"))')"
done
