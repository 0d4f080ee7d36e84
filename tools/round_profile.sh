#!/bin/bash
# Round evidence: bench JSON lines (bf16 headline, fp8 cfg5, train cfg3), rocprofv3 kernel trace +
# stats of the bf16 bench, PMC passes (separate runs): FETCH/WRITE for conv9 (bf16, fp8), lr,
# conv1, attn; SQ MFMA-busy group for the packed conv9 probe.
TAG=${1:-r1}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --dtype fp8 --cpu-baseline 0 > gpurun_out/$TAG/bench_fp8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/$TAG/bench_train.log 2>&1 || exit $?
PROBE_KERNELS="conv9 lr conv1 attn" bash tools/profile.sh $TAG || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d gpurun_out/prof_$TAG/pmc_conv9fp8_$C -o pmc --output-format csv -- \
    python3 tools/kernel_probe.py conv9 --dtype fp8 --reps 10 > gpurun_out/prof_$TAG/pmc_conv9fp8_$C.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -T -d gpurun_out/prof_$TAG/pmc_conv9_mfma -o pmc --output-format csv -- \
  python3 tools/kernel_probe.py conv9 --reps 10 > gpurun_out/prof_$TAG/pmc_conv9_mfma.log 2>&1 || exit $?
echo round profile done
