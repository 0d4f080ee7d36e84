#!/bin/bash
D=gpurun_out/smokeb2; mkdir -p $D
for V in "FS2_LIB=$PWD/oldlib/libfs2hip_prev.so" "FS2_CONV_NARROW=0" "FS2_LN_PAIRS=0" "FS2_CONV_SPLITK=0" "FS2_CONV_PHASED=0" "FS2_CONV_SPLITK=0 FS2_CONV_NARROW=0 FS2_LN_PAIRS=0 FS2_MEL_BF16=0"; do
  env $V timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/s.log 2>&1
  rc=$?
  echo "[$V] rc=$rc $(grep 'smoke\[bf16\]' $D/s.log)" >> $D/summary.txt
  [ $rc -ge 124 ] && exit $rc
done
exit 0
