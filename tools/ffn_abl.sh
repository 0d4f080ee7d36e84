#!/bin/bash
# Fused-FFN stall probe: the decoder-shape fused FFN timed (HIP events over graph replays) with the
# product library, with every weight load reading unit 0 (L1-resident: abl/libfs2hip_abl8.so,
# -DFFN_ABLATE=8) and with no weight loads (abl2). Built beforehand on the CPU side.
TAG=${1:-ffnabl}
O=gpurun_out/$TAG; mkdir -p $O
for lib in "" abl/libfs2hip_abl8.so abl/libfs2hip_abl2.so ""; do
  if [ -n "$lib" ]; then export FS2_LIB=$PWD/$lib FS2_LIB_ALLOW_MISSING=1; else unset FS2_LIB FS2_LIB_ALLOW_MISSING; fi
  timeout -k 10 120 python tools/kernel_probe.py ffn --time >> $O/ffn_time.log 2>&1 || { tail -5 $O/ffn_time.log; exit 1; }
  echo "lib=${lib:-product} $(tail -1 $O/ffn_time.log)"
done
