#!/bin/bash
# Round-end evidence: bench JSON line, rocprofv3 kernel trace + stats of the bench, PMC traffic
# passes for the decoder conv-k9 and the LR gather (separate runs, no trace domains).
TAG=${1:-r1}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || exit $?
PROBE_KERNELS="conv9 lr conv1 attn" bash tools/profile.sh $TAG || exit $?
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/$TAG/bench_train.log 2>&1 || exit $?
echo round profile done
