#!/bin/bash
# Vocoder-only profile: rocprofv3 kernel trace + stats of a short vocoder run (tools/kernel_probe-free).
O=gpurun_out/${1:-voc}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o voc --output-format csv -- \
  python3 tools/voc_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -3 $O/probe.log
