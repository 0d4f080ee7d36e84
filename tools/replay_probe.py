#!/usr/bin/env python3
"""Host cost of torch's CUDAGraph.replay() vs hipGraphLaunch on the same exec (bench forward)."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import bench
    from fs2amd.data import synth_batch, to_device
    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    batch = to_device(synth_batch(64, 64, seed=1), dev)
    with torch.no_grad():
        model(**batch)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s), torch.no_grad():
        model(**batch)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), torch.no_grad():
        model(**batch)
    g.replay()
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    ex = ctypes.c_void_p(g.raw_cuda_graph_exec())
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    K = 50
    for rep in range(3):
        t0 = time.perf_counter()
        hs = []
        for _ in range(K):
            a = time.perf_counter()
            g.replay()
            hs.append(time.perf_counter() - a)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(K):
            assert hip.hipGraphLaunch(ex, st) == 0
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"torch replay: {(t1 - t0) / K * 1e3:.4f} ms/step (host per call {sum(hs) / K * 1e3:.4f} ms); "
              f"hipGraphLaunch: {(t2 - t1) / K * 1e3:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
