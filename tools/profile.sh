#!/bin/bash
# rocprofv3 passes for one round: kernel trace + stats of the bench command, then separate PMC
# passes (FETCH_SIZE / WRITE_SIZE never in one pass; no trace domains beside --pmc).
# usage: tools/profile.sh <tag>      (run from the repo root on the GPU box)
set -u
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/bench_under_rocprof.log 2>&1 || exit $?
for K in ${PROBE_KERNELS:-conv9 lr}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_${K}_$C -o pmc --output-format csv -- \
      python3 tools/kernel_probe.py $K --reps 10 > $OUT/pmc_${K}_$C.log 2>&1 || exit $?
  done
done
echo profile done
