#!/bin/bash
# Split-hidden fused FFN: GPU tests, graph-timed probes (encoder / free-running decoder shapes,
# fused at (tile rows, nsplit) forms against the two launches), the free-running probe and a bench.
O=gpurun_out/${1:-ffnsplit}; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
for k in "enc_ffn --nsplit 4 --tile-rows 112" "enc_ffn --nsplit 1 --tile-rows 64" "enc_ffn --nsplit 2 --tile-rows 64" \
         "enc_ffn --nsplit 4 --tile-rows 64" "enc_ffn" "ffn_rows --nsplit 2 --tile-rows 112" "ffn_rows --nsplit 1 --tile-rows 64" \
         "ffn_rows --nsplit 2 --tile-rows 64" "ffn_rows --nsplit 4 --tile-rows 64" "ffn_rows" "ffn --tile-rows 64 --nsplit 1" "ffn"; do
  timeout -k 10 120 python tools/kernel_probe.py $k --time 2>&1 | tail -1 | sed "s/^/[$k] /" || exit 1
done
timeout -k 10 120 python tools/free_probe.py || exit 1
for V in 1 2; do
  timeout -k 10 300 python bench.py --extra 0 --vocoder 0 --cpu-baseline 0 --steps 30 > $O/bench_$V.log 2>&1 || { tail -20 $O/bench_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$V.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
done
