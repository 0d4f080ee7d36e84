#!/bin/bash
# A/B counters: phased 256x256 kernel on the conv9 shape at M=32768 (+ traffic passes for both).
FS2_CONV_PHASED=1 bash tools/pmc_cmd.sh c9_8p tools/m_sweep.py --ms 32768 --reps 5 || exit $?
