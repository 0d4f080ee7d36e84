#!/bin/bash
mkdir -p gpurun_out/epi4
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/epi4/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/epi4/summary.txt; [ $rc -gt 1 ] && exit $rc
for D in 0 2; do
  FS2_CONV_DEBUG=$D timeout -k 10 120 python tools/kernel_probe.py conv1 --time --reps 30 2>/dev/null | sed "s/^/new DBG=$D /" >> gpurun_out/epi4/summary.txt || exit $?
done
PROBES="conv1 enc_ln vp" bash tools/ab_lib.sh expressive-fastspeech2-mandarin_amd/fs2amd/_lib/libfs2hip_prev.so epi4 || exit $?
