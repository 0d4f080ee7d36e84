#!/bin/bash
# round-3 training checks: GPU train tests, bf16 full-size prints, train bench plain / DDP graphed,
# and the graphed train step once under rocprofv3 (the round-2 capture_end SIGSEGV case)
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_ref_checkpoint.py -q --timeout 200 --timeout-method thread -rf > $O/train_tests.log 2>&1; tail -3 $O/train_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -s -k "targets_bf16 or flip_rate or long_eval or targets_fp32" --timeout 200 --timeout-method thread -rf > $O/model_tests.log 2>&1; tail -2 $O/model_tests.log; grep -E "vs reference|free-running" $O/model_tests.log
timeout -k 10 200 python bench.py --mode train --graph 1 --steps 20 --warmup 5 > $O/train_graph.json 2>$O/train_graph.err && tail -1 $O/train_graph.json | cut -c1-300
timeout -k 10 200 python bench.py --mode train --graph 1 --ddp 1 --steps 20 --warmup 5 > $O/train_graph_ddp.json 2>$O/train_graph_ddp.err && tail -1 $O/train_graph_ddp.json | cut -c1-300
timeout -k 10 200 python bench.py --mode train --graph 0 --steps 10 --warmup 3 > $O/train_eager.json 2>$O/train_eager.err && tail -1 $O/train_eager.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train_graph -o run -- python3 bench.py --mode train --graph 1 --steps 5 --warmup 3 > $O/prof_train_graph.log 2>&1; echo "rocprof train graph rc=$?"; tail -2 $O/prof_train_graph.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -q --timeout 200 --timeout-method thread -rf > $O/graphs_tests.log 2>&1; tail -3 $O/graphs_tests.log
