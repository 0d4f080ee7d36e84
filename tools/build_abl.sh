#!/bin/bash
# analysis builds of the fused FFN: abl/libfs2hip_ab<bits>.so = the cached objects (FS2_OBJ_CACHE)
# with ffn.hip compiled under -DFFN_ABLATE=<bits> (bits: 1 no MFMAs, 2 no weight loads, 4 no reads)
set -e
C=${FS2_OBJ_CACHE:-/tmp/fs2obj}
CS=expressive-fastspeech2-mandarin_amd/csrc
mkdir -p abl
for b in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$CS -DFFN_ABLATE=$b -c $CS/ffn.hip -o /tmp/ffn_ab$b.o &
done
wait
for b in "$@"; do
  objs=$(ls $C/*.o | grep -v "/ffn.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfs2hip_ab$b.so $objs /tmp/ffn_ab$b.o
done
