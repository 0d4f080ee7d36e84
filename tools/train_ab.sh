#!/bin/bash
D=gpurun_out/trainab; mkdir -p $D
for i in 1 2; do
  for V in 0 1; do
    FS2_LN_PAIRS=$V timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $D/b.log 2>&1 || exit $?
    echo "LN_PAIRS=$V $(tail -n 1 $D/b.log | cut -c1-170)" >> $D/summary.txt
  done
done
