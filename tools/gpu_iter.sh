#!/bin/bash
# One GPU iteration: parity tests, per-kernel timings (HIP events), bench. Every GPU step has
# its own time limit; the script stops at the first crash/timeout (rc > 1 from pytest).
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $OUT/summary.txt
[ $rc -gt 1 ] && exit $rc
for K in ${PROBES:-conv9 conv1 qkv attn lr postnet enc_conv9 enc_ln vp}; do
  timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 20 >> $OUT/summary.txt 2>$OUT/probe_$K.err || { echo "probe $K failed rc=$?" >> $OUT/summary.txt; exit 3; }
done
timeout -k 10 500 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
echo "bench rc=$?" >> $OUT/summary.txt
tail -1 $OUT/bench.log >> $OUT/summary.txt
