#!/bin/bash
# fs2_hifigan_pair with waves as 4 channel pairs x 2 row halves (each B fragment feeds two MFMAs):
# vocoder tests + profile
O=gpurun_out/r5v3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoder.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/voc_tests.log 2>&1 || { tail -40 $O/voc_tests.log; exit 1; }
tail -3 $O/voc_tests.log
bash tools/prof_voc.sh r5v3/pair || exit 1
python3 tools/prof_summary.py $(ls gpurun_out/r5v3/pair/trace/*kernel_trace.csv | head -1) > $O/pair_kernels.txt
grep -h "vocoder bf16" $O/pair/probe.log
head -8 $O/pair_kernels.txt
