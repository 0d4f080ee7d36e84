#!/bin/bash
mkdir -p gpurun_out/attn2
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/attn2/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/attn2/summary.txt; [ $rc -gt 1 ] && exit $rc
PROBES="attn" bash tools/ab_lib.sh expressive-fastspeech2-mandarin_amd/fs2amd/_lib/libfs2hip_prev.so attn2 || exit $?
