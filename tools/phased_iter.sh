set -e
mkdir -p gpurun_out/ph1
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -q -p no:cacheprovider -k phased > gpurun_out/ph1/test.log 2>&1
timeout -k 10 200 python tools/m_sweep.py --ms 16384,24576,24883,27520,32768 > gpurun_out/ph1/sweep_default.txt 2>&1
FS2_CONV_PHASED=1 timeout -k 10 200 python tools/m_sweep.py --ms 16384,24576,24883,27520,32768 > gpurun_out/ph1/sweep_phased.txt 2>&1
FS2_CONV_PHASED=1 timeout -k 10 200 python tools/m_sweep.py --cin 512 --n 512 --ks 5 --ms 27520 > gpurun_out/ph1/sweep_phased_pn.txt 2>&1
timeout -k 10 200 python tools/m_sweep.py --cin 512 --n 512 --ks 5 --ms 27520 > gpurun_out/ph1/sweep_default_pn.txt 2>&1
