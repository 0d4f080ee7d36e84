#!/bin/bash
# fused-FFN ablation: time the kernel with analysis builds abl/libfs2hip_ab<bits>.so (FFN_ABLATE bits:
# 1 no MFMAs, 2 no weight-stage DMA, 4 no fragment reads)
mkdir -p gpurun_out/ffn_ab
for v in 0 "$@"; do
  if [ "$v" = 0 ]; then lib=""; else lib="FS2_LIB=abl/libfs2hip_ab$v.so"; fi
  echo "ablate=$v $(env $lib timeout -k 10 120 python tools/kernel_probe.py ffn --time --reps 20 2>&1 | tail -1)"
done | tee gpurun_out/ffn_ab/ablate.txt
