#!/bin/bash
# fused FFN timing at the cfg2 decoder shape, optionally A/B over env settings: tools/ffn_ab.sh [tag]
mkdir -p gpurun_out/ffn_ab
echo "$(timeout -k 10 120 python tools/kernel_probe.py ffn --time --reps 20 2>&1 | tail -1)" > gpurun_out/ffn_ab/${1:-base}.txt
cat gpurun_out/ffn_ab/${1:-base}.txt
