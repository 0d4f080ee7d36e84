#!/bin/bash
# One GPU checkpoint of the tree: the GPU suite + the driver-protocol bench line (gpu_check.sh),
# smoke(), a rocprofv3 kernel trace of the bench (graph-replayed forward table) and the PMC
# passes over eager forwards (per-launch HBM bytes / MFMA busy). SKIP_TESTS=1, SKIP_TRACE=1,
# SKIP_FREE=1 (free-running timing + trace), SKIP_PMC=1 drop parts. Every GPU step has its own time limit; stop at the first failure.
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  bash tools/gpu_check.sh $TAG || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
else
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-300
fi
if [ -z "${SKIP_TRACE:-}" ]; then
  bash tools/fwd_trace.sh $TAG/trace_run || exit 1
fi
if [ -z "${SKIP_FREE:-}" ]; then
  timeout -k 10 120 python3 tools/free_probe.py --eager > $O/free_eager.log 2>&1 || { tail -20 $O/free_eager.log; exit 1; }
  tail -1 $O/free_eager.log
  bash tools/free_trace.sh $TAG/free || exit 1
fi
if [ -z "${SKIP_PMC:-}" ]; then
  bash tools/pmc_fwd.sh $TAG ${PMC_ARGS:-} || exit 1
fi
