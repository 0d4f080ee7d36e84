#!/bin/bash
mkdir -p gpurun_out/epi2
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/epi2/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/epi2/summary.txt; [ $rc -gt 1 ] && exit $rc
PROBES="conv1 qkv" bash tools/ab_lib.sh expressive-fastspeech2-mandarin_amd/fs2amd/_lib/libfs2hip_prev.so epi2 || exit $?
bash tools/pmc_cmd.sh conv1_ring tools/kernel_probe.py conv1 --reps 5 || exit $?
