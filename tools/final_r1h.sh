#!/bin/bash
# round-end evidence: full GPU test suite, smoke, then the round profile (bench lines, kernel trace, PMC)
mkdir -p gpurun_out/r1h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r1h/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1h/smoke.log 2>&1 || exit $?
bash tools/round_profile2.sh r1h
