#!/bin/bash
# One rocprofv3 kernel trace of the headline bench (no extra workloads), then the per-launch table
# of one graph-replayed forward (tools/fwd_gaps.py).
O=gpurun_out/${1:-fwdtrace}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 tools/fwd_gaps.py $(ls $O/trace/*kernel_trace.csv | head -1) > $O/forward_kernels.txt
tail -1 $O/bench.log | cut -c1-200
tail -3 $O/forward_kernels.txt
