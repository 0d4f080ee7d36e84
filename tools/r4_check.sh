#!/bin/bash
# Round-4 GPU check: focused kernel tests, forward / vocoder / train profiles (train with the
# per-op path and with the fused training nodes), then the whole GPU suite and the bench line.
# Plain test failures (pytest exit 1) do not stop the profiles; a crash, abort or time limit does.
TAG=${1:-r4}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest $FOCUS -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/first.log 2>&1
rc=$?
tail -3 $O/first.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "focused tests ended with $rc: stopping"; exit $rc; fi
bash tools/fwd_trace.sh $TAG && bash tools/prof_voc.sh $TAG || exit 1
FS2_TRAIN_FUSED=0 FS2_LOSS_FUSED=0 GRAPH=1 bash tools/prof_train.sh ${TAG}_train_old || exit 1
GRAPH=1 bash tools/prof_train.sh ${TAG}_train || exit 1
[ $rc -eq 0 ] || exit 1
bash tools/gpu_check.sh $TAG
