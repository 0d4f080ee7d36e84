#!/bin/bash
mkdir -p gpurun_out/trprof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trprof/trace -o tr --output-format csv -- python3 bench.py --mode train --steps 5 --warmup 2 > gpurun_out/trprof/log.txt 2>&1 || exit $?
