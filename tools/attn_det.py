#!/usr/bin/env python3
"""Attention determinism probe: the bf16 attention on packed free-running-like rows, eager x3 and
graph-replayed x3, all compared bit for bit with the first eager run."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
import torch  # noqa: E402


def main():
    from fs2amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(60, 300, (64,), generator=g)
    lens[3] = 960
    T = 960
    lay = ops.SeqLayout(lens.to(dev), T)
    qkv = (torch.randn(lay.capacity, 768, generator=g) * 0.5).to(dev, torch.bfloat16)
    ref = ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay).clone()
    R = int(lay.cu[-1])
    bad = 0
    for i in range(3):
        o = ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)
        bad += int((o[:R] != ref[:R]).any())
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            og = ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)
    torch.cuda.current_stream(dev).wait_stream(s)
    gbad = 0
    for i in range(3):
        gr.replay()
        torch.cuda.synchronize()
        d = (og[:R].float() - ref[:R].float()).abs()
        gbad += int((og[:R] != ref[:R]).any())
        print("graph replay", i, "max diff", float(d.max()), "rows differing", int((d.amax(1) > 0).sum()))
    print("eager mismatches", bad, "graph mismatches", gbad)


if __name__ == "__main__":
    main()
