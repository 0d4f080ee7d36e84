#!/bin/bash
# Round-3 (late) evidence: full bench line (headline + extras + CPU baseline), rocprofv3 kernel
# trace + stats of the bench, FETCH/WRITE passes of the fused FFN, SQ counters of attention and the
# fused FFN, the free-running cfg2 trace, the graphed cfg3 train line.
TAG=${1:-r3d}
O=gpurun_out/prof_$TAG; mkdir -p gpurun_out/$TAG $O
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 > gpurun_out/$TAG/bench_train.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/trace -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra 0 --vocoder 0 > $O/bench_under_rocprof.log 2>&1 || exit $?
python3 tools/fwd_gaps.py $(ls $O/trace/*kernel_trace.csv | head -1) > $O/forward_kernels.txt
tail -1 $O/forward_kernels.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $O/pmc_ffn_$C -o pmc --output-format csv -- \
    python3 tools/kernel_probe.py ffn --reps 10 > $O/pmc_ffn_$C.log 2>&1 || exit $?
done
for K in attn ffn; do
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/pmc_${K}_sq -o pmc --output-format csv -- \
    python3 tools/kernel_probe.py $K --reps 10 > $O/pmc_${K}_sq.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/free -o free --output-format csv -- \
  python3 tools/free_probe.py > $O/free.log 2>&1 || exit $?
python3 tools/fwd_gaps.py $(ls $O/free/*kernel_trace.csv | head -1) > $O/free_kernels.txt
tail -1 $O/free.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/$TAG/smoke.log
echo round profile done
