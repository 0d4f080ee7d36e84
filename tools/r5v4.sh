#!/bin/bash
# fs2_hifigan_pair generalised to C = 64 (512-sample tiles, 128-byte rows): vocoder tests, then the
# vocoder profile with the 64-channel stage as the MRF launch (default) and as 9 pair launches
O=gpurun_out/r5v4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoder.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/voc_tests.log 2>&1 || { tail -40 $O/voc_tests.log; exit 1; }
tail -2 $O/voc_tests.log
bash tools/prof_voc.sh r5v4/mrf64 || exit 1
FS2_VOC_PAIR64=1 bash tools/prof_voc.sh r5v4/pair64 || exit 1
for v in mrf64 pair64; do python3 tools/prof_summary.py $(ls gpurun_out/r5v4/$v/trace/*kernel_trace.csv | head -1) > $O/${v}_kernels.txt; grep -h "vocoder bf16" $O/$v/probe.log; head -6 $O/${v}_kernels.txt; done
