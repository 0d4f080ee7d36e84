#!/bin/bash
# Checkpoint: the whole GPU suite + the default bench line (tools/gpu_check.sh), smoke(), and the
# graphed training bench line. Each GPU step has its own time limit; stop at the first failure.
TAG=${1:-r4l}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --mode train --graph 1 --steps 20 --warmup 5 > $O/train_graph.log 2>&1 || { tail -20 $O/train_graph.log; exit 1; }
tail -1 $O/train_graph.log | cut -c1-300
