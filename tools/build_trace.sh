#!/bin/bash
# analysis builds of the fused FFN with per-phase clock stamps: abl/libfs2hip_trace.so, plus
# abl/libfs2hip_trace_e<bits>.so for each argument (LN epilogue ablation bits, conv_common.h dbg)
set -e
C=${FS2_OBJ_CACHE:-/tmp/fs2obj}
CS=expressive-fastspeech2-mandarin_amd/csrc
mkdir -p abl
OBJS=$(ls $C/*.o | grep -v "/ffn.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$CS -DFFN_TRACE=1 -c $CS/ffn.hip -o /tmp/ffn_trace.o &
for e in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$CS -DFFN_TRACE=1 -DFFN_EPI_DBG=$e -c $CS/ffn.hip -o /tmp/ffn_trace_e$e.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfs2hip_trace.so $OBJS /tmp/ffn_trace.o
for e in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfs2hip_trace_e$e.so $OBJS /tmp/ffn_trace_e$e.o
done
