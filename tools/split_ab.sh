D=gpurun_out/split1; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_packed.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $D/t.log 2>&1 || exit $?
for V in "FS2_CONV_PHASED=0" "FS2_CONV_PHASED=1"; do
  env $V timeout -k 10 200 python tools/m_sweep.py --ms 8576,16384,24576,24883,25600,27520,32768 --reps 30 > $D/s.txt 2>&1 || exit $?
  echo "$V $(grep M= $D/s.txt | awk '{print $2, $3}' | tr '\n' ' ')" >> $D/summary.txt
done
bash tools/ab_multi.sh split1ab "FS2_CONV_PHASED=0" "FS2_CONV_PHASED=1"
