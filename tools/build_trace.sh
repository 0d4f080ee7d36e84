#!/bin/bash
# analysis builds of the fused FFN with per-phase clock stamps: abl/libfs2hip_trace.so, plus one
# library per argument: e<bits> -> abl/libfs2hip_trace_e<bits>.so (LN epilogue ablation bits,
# conv_common.h dbg), a<bits> -> abl/libfs2hip_trace_a<bits>.so (FFN_ABLATE bits)
set -e
C=${FS2_OBJ_CACHE:-/tmp/fs2obj}
CS=expressive-fastspeech2-mandarin_amd/csrc
mkdir -p abl
OBJS=$(ls $C/*.o | grep -v "/ffn.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$CS -DFFN_TRACE=1 -c $CS/ffn.hip -o /tmp/ffn_trace.o &
for v in "$@"; do
  case $v in
    e*) F="-DFFN_EPI_DBG=${v#e}" ;;
    a*) F="-DFFN_ABLATE=${v#a}" ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$CS -DFFN_TRACE=1 $F -c $CS/ffn.hip -o /tmp/ffn_trace_$v.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfs2hip_trace.so $OBJS /tmp/ffn_trace.o
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfs2hip_trace_$v.so $OBJS /tmp/ffn_trace_$v.o
done
