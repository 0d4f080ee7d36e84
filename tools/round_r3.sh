#!/bin/bash
# Round-3 evidence: bench line (bf16 headline + extras + CPU baseline), rocprofv3 kernel trace +
# stats of the bench, PMC FETCH/WRITE passes (separate runs) of the fused FFN and the other ops,
# an SQ pass on the fused FFN, the cfg3 train line (graphed) and its kernel trace.
TAG=${1:-r3a}
O=gpurun_out/prof_$TAG; mkdir -p gpurun_out/$TAG $O
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 > gpurun_out/$TAG/bench_train.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra 0 --vocoder 0 > $O/bench_under_rocprof.log 2>&1 || exit $?
for K in ffn attn fc qkv lr; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C -T -d $O/pmc_${K}_$C -o pmc --output-format csv -- \
      python3 tools/kernel_probe.py $K --reps 10 > $O/pmc_${K}_$C.log 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/pmc_ffn_sq -o pmc --output-format csv -- \
  python3 tools/kernel_probe.py ffn --reps 10 > $O/pmc_ffn_sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/train -o train --output-format csv -- \
  python3 bench.py --mode train --graph 1 --steps 5 --warmup 3 > $O/train_under_rocprof.log 2>&1 || exit $?
echo round profile done
