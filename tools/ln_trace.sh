#!/bin/bash
# kernel-trace durations of the LN-epilogue GEMMs under FS2_CONV_DEBUG ablations
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
D=gpurun_out/lntrace; mkdir -p $D
for K in fc conv1; do
  for V in 0 1 2 3; do
    FS2_CONV_DEBUG=$V timeout -k 10 120 rocprofv3 --kernel-trace -d $D/${K}_$V -o t --output-format csv -- python3 tools/kernel_probe.py $K --time --reps 30 > $D/${K}_$V.log 2>&1 || exit $?
  done
done
