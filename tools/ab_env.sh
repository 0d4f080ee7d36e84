#!/bin/bash
# A/B one env switch on one box: alternating m_sweep runs and bench runs.  usage: ab_env.sh VAR tag
V=$1; TAG=$2
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  for X in 1 0; do
    env $V=$X timeout -k 10 200 python tools/m_sweep.py --ms ${MS:-24883,27520} --reps 30 > gpurun_out/$TAG/sweep_${X}_$i.txt 2>&1 || exit $?
    echo "$V=$X run$i $(grep M= gpurun_out/$TAG/sweep_${X}_$i.txt | tr '\n' ' ')" >> gpurun_out/$TAG/summary.txt
  done
done
for X in 1 0 1 0; do
  env $V=$X timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/$TAG/bench_$X.log 2>&1 || exit $?
  echo "$V=$X bench $(tail -1 gpurun_out/$TAG/bench_$X.log | cut -c80-140)" >> gpurun_out/$TAG/summary.txt
done
