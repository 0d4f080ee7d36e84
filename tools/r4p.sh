#!/bin/bash
# Round-4 final checkpoint: the GPU suite + default bench line, smoke(), the graphed training line,
# a forward trace (graph replays) and vocoder profile, and the PMC counter passes of the 32-query
# attention. Each GPU step has its own time limit; stop at the first failure.
TAG=${1:-r4p}
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --mode train --graph 1 --steps 20 --warmup 5 > $O/train_graph.log 2>&1 || { tail -20 $O/train_graph.log; exit 1; }
tail -1 $O/train_graph.log | cut -c1-200
bash tools/fwd_trace.sh $TAG/trace_run && bash tools/prof_voc.sh $TAG || exit 1
bash tools/pmc_cmd.sh ${TAG}_attn tools/kernel_probe.py attn --reps 10 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_attn attn32 > $O/pmc_attn32.txt
tail -12 $O/pmc_attn32.txt
