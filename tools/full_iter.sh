#!/bin/bash
# full GPU suite + default bf16 bench (one box)
D=gpurun_out/${1:-full}; mkdir -p $D
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log > $D/summary.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $D/bench.log 2>&1 || exit $?
tail -1 $D/bench.log >> $D/summary.txt
