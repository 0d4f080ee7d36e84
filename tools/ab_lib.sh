#!/bin/bash
# A/B two builds of libfs2hip on one box (FS2_LIB override), alternating.  usage: ab_lib.sh B.so tag
ALT=$1; TAG=$2
mkdir -p gpurun_out/$TAG
CUR=expressive-fastspeech2-mandarin_amd/fs2amd/_lib/libfs2hip.so
for i in 1 2; do
  for L in $CUR $ALT; do
    n=$(basename $L .so)
    for K in ${PROBES:-conv1 enc_ln qkv conv9}; do
      FS2_LIB=$PWD/$L timeout -k 10 120 python tools/kernel_probe.py $K --time --reps 30 2>/dev/null | sed "s/^/$n run$i /" >> gpurun_out/$TAG/summary.txt || exit $?
    done
    FS2_LIB=$PWD/$L timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/$TAG/bench_${n}_$i.log 2>&1 || exit $?
    echo "$n run$i bench $(tail -1 gpurun_out/$TAG/bench_${n}_$i.log | cut -c80-120)" >> gpurun_out/$TAG/summary.txt
  done
done
