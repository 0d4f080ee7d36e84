#!/bin/bash
# cfg3 train-step profile: rocprofv3 kernel trace + stats of a short `bench.py --mode train` run.
O=gpurun_out/${1:-trainprof}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o train --output-format csv -- \
  python3 bench.py --mode train --steps 5 --warmup 2 --graph ${GRAPH:-0} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
