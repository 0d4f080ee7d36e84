#!/bin/bash
# torch.library ops on the GPU, then the whole GPU suite once more on the final tree.
TAG=${1:-r4r}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_library.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/library.log 2>&1 || { tail -40 $O/library.log; exit 1; }
tail -3 $O/library.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
