#!/bin/bash
# default 8 column waves: the whole GPU suite + smoke, then a bench line
D=gpurun_out/w8full; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > $D/bench.log 2>&1
