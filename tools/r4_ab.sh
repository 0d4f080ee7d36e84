#!/bin/bash
# Round-4 A/B: the attention / vocoder / graph / Adam tests, attention timing in both forms
# (FS2_ATTN32=1/0), the VariancePredictor sets with the L2 warm-up on / off (warm and after a 512 MB
# flush), a vocoder profile and a forward trace. Each GPU step has its own time limit; stop at the
# first failure.
TAG=${1:-ab}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_vocoder.py tests/test_gpu_train.py tests/test_gpu_graphs.py -k "vocoder or mrf or generator or attention or attn or graph" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_train_kernels.py -k adam -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_adam.log 2>&1 || { tail -20 $O/tests_adam.log; exit 1; }
tail -1 $O/tests_adam.log
for v in 1 0 1 0; do
  FS2_ATTN32=$v timeout -k 10 120 python tools/kernel_probe.py attn --time >> $O/attn_time.log 2>&1 || { tail -5 $O/attn_time.log; exit 1; }
  echo "attn32=$v $(tail -1 $O/attn_time.log)"
done
for pf in 1 0; do for k in vpf_dp vpf_en; do for fl in 0 512; do
  FS2_VP_PREFETCH=$pf timeout -k 10 120 python tools/kernel_probe.py $k --time --reps 10 --flush $fl >> $O/vp_time.log 2>&1 || { tail -5 $O/vp_time.log; exit 1; }
  echo "prefetch=$pf $(tail -1 $O/vp_time.log)"
done; done; done
bash tools/ffn_abl.sh $TAG || exit 1
for v in 0 1 0 1; do
  FS2_FFN_ACQUIRE=$v timeout -k 10 120 python tools/kernel_probe.py enc_ffn --time >> $O/enc_ffn_time.log 2>&1 || { tail -5 $O/enc_ffn_time.log; exit 1; }
  echo "ffn_acquire=$v $(tail -1 $O/enc_ffn_time.log)"
done
bash tools/prof_voc.sh $TAG && bash tools/fwd_trace.sh $TAG
