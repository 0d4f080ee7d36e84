#!/bin/bash
# kernel trace of the bench (graph replay), for per-forward gap / duration analysis
D=gpurun_out/${1:-trace}; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $D/t -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $D/b.log 2>&1
