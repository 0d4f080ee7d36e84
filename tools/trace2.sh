#!/bin/bash
# rocprofv3 kernel traces of (1) the headline bench forward and (2) free-running cfg2 synthesis
# (SynthGraphs), each reduced to the per-launch table of one forward (tools/fwd_gaps.py).
O=gpurun_out/${1:-trace2}; mkdir -p $O; export TMPDIR=/tmp
bash tools/fwd_trace.sh ${1:-trace2}/bench || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/free -o free --output-format csv -- \
  python3 tools/free_probe.py > $O/free.log 2>&1 || { tail -20 $O/free.log; exit 1; }
python3 tools/fwd_gaps.py $(ls $O/free/*kernel_trace.csv | head -1) > $O/free_kernels.txt
tail -2 $O/free.log; tail -1 $O/free_kernels.txt
