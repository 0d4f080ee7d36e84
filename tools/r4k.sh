#!/bin/bash
# Attention forms (FS2_ATTN32_FORM 4x2 / 8x2 / 8x3, FS2_ATTN32=0) and write-through output stores
# (FS2_OUT_SC1): the attention tests under each form, standalone timing, and a forward trace with
# and without sc1 stores. Each GPU step has its own time limit; stop at the first failure.
TAG=${1:-r4k}
O=gpurun_out/$TAG; mkdir -p $O
T="tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_train.py"
for f in 4x2 8x2 8x3; do
  FS2_ATTN32_FORM=$f timeout -k 10 300 python -u -m pytest $T -k "attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$f.log 2>&1 || { tail -20 $O/tests_$f.log; exit 1; }
  echo "form $f: $(tail -1 $O/tests_$f.log)"
done
FS2_OUT_SC1=1 timeout -k 10 400 python -u -m pytest $T tests/test_gpu_graphs.py -k "attention or ffn or graph" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_sc1.log 2>&1 || { tail -20 $O/tests_sc1.log; exit 1; }
echo "sc1: $(tail -1 $O/tests_sc1.log)"
for f in 4x2 8x2 8x3 old nostage 4x2 8x2 8x3 old nostage; do
  a=1; st=1
  if [ $f = old ]; then a=0; fi
  if [ $f = nostage ]; then st=0; fi
  FS2_ATTN32=$a FS2_ATTN_OSTAGE=$st FS2_ATTN32_FORM=$f timeout -k 10 120 python tools/kernel_probe.py attn --time >> $O/attn_time.log 2>&1 || { tail -5 $O/attn_time.log; exit 1; }
  echo "form=$f $(tail -1 $O/attn_time.log)"
done
FS2_OUT_SC1=1 bash tools/fwd_trace.sh $TAG/sc1 || exit 1
bash tools/fwd_trace.sh $TAG/plain || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
