#!/usr/bin/env python3
"""Capture the bench forward as a HIP graph and dump its nodes (DOT) to gpurun_out/graph/."""
import os
import sys

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
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s), torch.no_grad():
        model(**batch)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    g.enable_debug_mode()
    with torch.cuda.graph(g), torch.no_grad():
        model(**batch)
    os.makedirs("gpurun_out/graph", exist_ok=True)
    g.debug_dump("gpurun_out/graph/fwd.dot")
    print("dumped")


if __name__ == "__main__":
    main()
