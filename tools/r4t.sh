#!/bin/bash
# Split-hidden FFN L2 warm-up (FS2_FFN_PREFETCH=1): FFN tests under it, the encoder FFN probe
# (cold after a 512 MB flush, and warm) with it on / off, and a forward trace with it on.
TAG=${1:-r4t}
O=gpurun_out/$TAG; mkdir -p $O
FS2_FFN_PREFETCH=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for pf in 0 1; do for fl in 512 0; do
  FS2_FFN_PREFETCH=$pf timeout -k 10 120 python tools/kernel_probe.py enc_ffn --time --flush $fl >> $O/enc.log 2>&1 || { tail -5 $O/enc.log; exit 1; }
  echo "prefetch=$pf flush=$fl $(tail -1 $O/enc.log)"
done; done; done
FS2_FFN_PREFETCH=1 bash tools/fwd_trace.sh $TAG/pf || exit 1
bash tools/fwd_trace.sh $TAG/nopf || exit 1
for t in pf nopf; do echo "$t: $(grep ffn_fused $O/$t/forward_kernels.txt | head -4 | awk '{printf "%s ", $(NF-2)}') $(tail -1 $O/$t/forward_kernels.txt | cut -c1-60)"; done
