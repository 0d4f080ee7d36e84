#!/bin/bash
# kernel trace of the bench with / without the bf16 mel copy (per-kernel deltas)
D=gpurun_out/melbftr; mkdir -p $D
export TMPDIR=/tmp
for V in 0 1; do
  FS2_MEL_BF16=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $D/t$V -o bench --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $D/b$V.log 2>&1 || exit $?
done
