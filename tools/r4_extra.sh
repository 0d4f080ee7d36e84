#!/bin/bash
# Training bench lines (graphed; graphed + in-graph RCCL all-reduce) and PMC counter passes for the
# attention and fused-FFN kernels (kernel_probe.py shapes = the cfg2 decoder).
TAG=${1:-r4x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python bench.py --mode train --graph 1 --steps 20 --warmup 5 > $O/train_graph.log 2>&1 || { tail -20 $O/train_graph.log; exit 1; }
tail -1 $O/train_graph.log | cut -c1-300
timeout -k 10 300 python bench.py --mode train --graph 1 --ddp 1 --steps 20 --warmup 5 > $O/train_graph_ddp.log 2>&1 || { tail -20 $O/train_graph_ddp.log; exit 1; }
tail -1 $O/train_graph_ddp.log | cut -c1-300
timeout -k 10 300 python bench.py --mode train --graph 0 --steps 10 --warmup 3 > $O/train_eager.log 2>&1 || { tail -20 $O/train_eager.log; exit 1; }
tail -1 $O/train_eager.log | cut -c1-300
bash tools/pmc_cmd.sh ${TAG}_attn tools/kernel_probe.py attn --reps 10 || exit 1
bash tools/pmc_cmd.sh ${TAG}_ffn tools/kernel_probe.py ffn --reps 10 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_attn attn_bf16 > $O/pmc_attn.txt
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_ffn ffn_fused > $O/pmc_ffn.txt
cat $O/pmc_attn.txt | tail -8
