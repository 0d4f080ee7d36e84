mkdir -p gpurun_out/ring9

for V in "FS2_CONV_RING9=0" "FS2_CONV_RING9=1" "FS2_CONV_RING9=1 FS2_CONV_SPLITK=0" "FS2_CONV_PHASED=1"; do
  env $V timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576,24883,25600,27520,32768 --reps 30 > gpurun_out/ring9/s.txt 2>&1 || exit $?
  echo "$V $(grep M= gpurun_out/ring9/s.txt | awk '{print $2, $3}' | tr '\n' ' ')" >> gpurun_out/ring9/summary.txt
done
