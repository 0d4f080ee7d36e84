#!/bin/bash
# One GPU call = one tag + a list of steps, run in order; every GPU step has its own time limit and
# the chain stops at the first failure (no GPU step after a fault / abort / timeout).
#   bash tools/run.sh TAG STEP [STEP ...]
# steps:
#   tests[=PYTEST_TARGETS]  pytest -m gpu (default: the whole tests/ dir; comma-separated targets, e.g.
#                           tests=tests/test_gpu_ops.py,tests/test_gpu_ffn.py)
#   smoke                   __graft_entry__.smoke()
#   bench                   the default bench line (50 / 20, all extra keys)
#   driver                  the driver's protocol: --gpus 1 --steps 20 --warmup 5
#   train                   bench.py --mode train --graph 1 (cfg3 line)
#   free / free_eager       tools/free_probe.py (SynthGraphs / eager), 8 distinct batches
#   fwd_trace               rocprofv3 kernel trace of the bench -> forward_kernels.txt
#   free_trace              rocprofv3 kernel trace of the free-running loop -> free_kernels.txt
#   train_trace             rocprofv3 kernel trace of the graphed cfg3 step -> train_steps.txt
#   voc                     rocprofv3 kernel trace of the vocoder probe -> voc_kernels.txt
#   pmc                     PMC passes over eager forwards (tools/pmc_fwd.sh)
#   attn_abl                tools/attn_abl.py run (build the tracelib/ variants first)
#   probe:ARGS              python tools/kernel_probe.py ARGS (colons in ARGS become spaces)
# Environment variables set on the call (FS2_*) apply to every step.
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
fail() { tail -${2:-30} $1; exit 1; }
for st in "$@"; do
  case $st in
    tests|tests=*)
      T=${st#tests}; T=${T#=}; T=${T:-tests}; T=${T//,/ }
      timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        > $O/tests.log 2>&1 || fail $O/tests.log 40
      tail -2 $O/tests.log ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || fail $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || fail $O/bench.log
      tail -1 $O/bench.log | cut -c1-300 ;;
    driver)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || fail $O/bench_driver.log
      tail -1 $O/bench_driver.log | cut -c1-300 ;;
    train)
      timeout -k 10 400 python bench.py --mode train --graph 1 > $O/train.log 2>&1 || fail $O/train.log
      grep -h '"metric"' $O/train.log | cut -c1-260 ;;
    free)
      timeout -k 10 200 python tools/free_probe.py > $O/free.log 2>&1 || fail $O/free.log 20
      grep -v amdgpu.ids $O/free.log | tail -1 ;;
    free_eager)
      timeout -k 10 200 python tools/free_probe.py --eager > $O/free_eager.log 2>&1 || fail $O/free_eager.log 20
      grep -v amdgpu.ids $O/free_eager.log | tail -1 ;;
    fwd_trace) bash tools/fwd_trace.sh $TAG/fwd || exit 1 ;;
    free_trace) bash tools/free_trace.sh $TAG/free || exit 1 ;;
    train_trace)
      GRAPH=1 bash tools/prof_train.sh $TAG/ttr || exit 1
      python3 tools/train_steps.py $O/ttr/trace/train_kernel_trace.csv > $O/train_steps.txt
      head -12 $O/train_steps.txt ;;
    voc)
      bash tools/prof_voc.sh $TAG/voc || exit 1
      python3 tools/prof_summary.py $(ls $O/voc/trace/*kernel_trace.csv | head -1) > $O/voc_kernels.txt
      head -8 $O/voc_kernels.txt ;;
    pmc) bash tools/pmc_fwd.sh $TAG > $O/pmc.log 2>&1 || fail $O/pmc.log 20 ;;
    attn_abl)
      timeout -k 10 600 python tools/attn_abl.py run > $O/attn_abl.log 2>&1 || fail $O/attn_abl.log
      cat $O/attn_abl.log ;;
    probe:*)
      A=${st#probe:}; A=${A//:/ }
      N=$(echo $A | tr ' ' '_')
      timeout -k 10 200 python tools/kernel_probe.py $A > $O/probe_$N.log 2>&1 || fail $O/probe_$N.log 20
      grep -v amdgpu.ids $O/probe_$N.log | tail -3 ;;
    *) echo "run.sh: unknown step $st"; exit 2 ;;
  esac
done
