#!/bin/bash
# Round evidence (defaults): bench JSON lines (bf16 headline, fp8 cfg5, train cfg3), rocprofv3
# kernel trace + stats of the bf16 bench, PMC FETCH/WRITE passes (separate runs) per op probe,
# SQ MFMA group for conv9.
TAG=${1:-r1e}
O=gpurun_out/prof_$TAG; mkdir -p gpurun_out/$TAG $O
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --dtype fp8 --cpu-baseline 0 > gpurun_out/$TAG/bench_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/$TAG/bench_train.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $O/bench_under_rocprof.log 2>&1 || exit $?
for K in conv9 lr lr4 attn conv1 fc qkv; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C -T -d $O/pmc_${K}_$C -o pmc --output-format csv -- \
      python3 tools/kernel_probe.py $K --reps 10 > $O/pmc_${K}_$C.log 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -T -d $O/pmc_conv9_mfma -o pmc --output-format csv -- \
  python3 tools/kernel_probe.py conv9 --reps 10 > $O/pmc_conv9_mfma.log 2>&1 || exit $?
echo round profile done
