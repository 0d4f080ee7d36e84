#!/bin/bash
# Round evidence (one call): bench JSON lines (bf16 headline with extras, fp8 cfg5, train cfg3),
# rocprofv3 kernel trace + stats of the bf16 bench (one graph-replayed forward kernel by kernel),
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) per op probe, SQ MFMA group on the conv-k9 probe.
TAG=${1:-r2}
O=gpurun_out/$TAG; P=$O/prof; mkdir -p $O $P
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --dtype fp8 --cpu-baseline 0 --extra 0 --vocoder 0 > $O/bench_fp8.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $O/bench_train.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra 0 --vocoder 0 > $P/bench_under_rocprof.log 2>&1 || exit 1
python3 tools/fwd_gaps.py $(ls $P/trace/*kernel_trace.csv | head -1) > $O/forward_kernels.txt
python3 tools/prof_summary.py $(ls $P/trace/*kernel_trace.csv | head -1) > $O/kernel_summary.txt
for K in conv9 qkv lr fc conv1 attn; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $C -d $P/pmc_${K}_$C -o pmc --output-format csv -- \
      python3 tools/kernel_probe.py $K --reps 10 > $P/pmc_${K}_$C.log 2>&1 || exit 1
  done
done
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $P/pmc_conv9_mfma \
  -o pmc --output-format csv -- python3 tools/kernel_probe.py conv9 --reps 10 > $P/pmc_conv9_mfma.log 2>&1 || exit 1
echo round profile done
