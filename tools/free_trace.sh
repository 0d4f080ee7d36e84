#!/bin/bash
# rocprofv3 kernel trace of the free-running synthesis loop (tools/free_probe.py, SynthGraphs or
# --eager) and the per-launch table of one call (tools/fwd_gaps.py, calls cut at cond_kernel).
O=gpurun_out/${1:-freetrace}; shift; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o free --output-format csv -- \
  python3 tools/free_probe.py "$@" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 tools/fwd_gaps.py $(ls $O/trace/*kernel_trace.csv | head -1) --start cond_kernel > $O/free_kernels.txt
tail -1 $O/probe.log; tail -2 $O/free_kernels.txt
