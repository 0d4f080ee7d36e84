#!/bin/bash
# Free-running cfg2 A/B: attention form by sequence length (default) vs forced 8x2, write-through
# stores on / off; eager and SynthGraphs. Then the attention tests under the default rule.
TAG=${1:-r4m}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_model.py -k "attention or free or packed" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in "default" "FS2_ATTN32_FORM=8x2" "FS2_OUT_SC1=0" "FS2_ATTN32_FORM=4x2 FS2_OUT_SC1=0"; do
  for m in --eager ""; do
    env $( [ "$v" = default ] || echo $v ) timeout -k 10 120 python tools/free_probe.py $m >> $O/free.log 2>&1 || { tail -5 $O/free.log; exit 1; }
    echo "$v $m: $(tail -1 $O/free.log)"
  done
done
done
