#!/bin/bash
# One GPU check: optional focused tests (FIRST_TESTS), the GPU test suite, then the default bench
# line. Every GPU step has its own time limit and the chain stops at the first failure.
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "${FIRST_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest $FIRST_TESTS ${FIRST_K:+-k "$FIRST_K"} -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $O/first.log 2>&1 || { tail -40 $O/first.log; exit 1; }
  tail -3 $O/first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_ARGS:-} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
