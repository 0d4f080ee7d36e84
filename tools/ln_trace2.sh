#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
D=gpurun_out/lntrace2; mkdir -p $D
for V in 1 5 9 17 29 3; do
  FS2_CONV_DEBUG=$V timeout -k 10 120 rocprofv3 --kernel-trace -d $D/fc_$V -o t --output-format csv -- python3 tools/kernel_probe.py fc --time --reps 30 > $D/fc_$V.log 2>&1 || exit $?
done
