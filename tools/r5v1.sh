#!/bin/bash
# fs2_hifigan_pair (the 128-channel stage, one launch per ResBlock1 dilation pair): vocoder tests,
# then the vocoder profile with the pair path and the per-conv path (FS2_VOC_PAIR=0) for A/B
O=gpurun_out/r5v1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoder.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/voc_tests.log 2>&1 || { tail -40 $O/voc_tests.log; exit 1; }
tail -3 $O/voc_tests.log
bash tools/prof_voc.sh r5v1/pair || exit 1
python3 tools/prof_summary.py $(ls gpurun_out/r5v1/pair/trace/*kernel_trace.csv | head -1) > $O/pair_kernels.txt
FS2_VOC_PAIR=0 bash tools/prof_voc.sh r5v1/perconv || exit 1
python3 tools/prof_summary.py $(ls gpurun_out/r5v1/perconv/trace/*kernel_trace.csv | head -1) > $O/perconv_kernels.txt
head -12 $O/pair_kernels.txt
