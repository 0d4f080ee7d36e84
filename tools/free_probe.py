#!/usr/bin/env python3
"""Free-running cfg2 synthesis (SynthGraphs) repeated, for rocprofv3 kernel traces: the bench's
free_running_cfg2 leg alone. --eager: the eager forward instead."""
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
    from fs2amd.graphs import SynthGraphs

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    b = to_device(synth_batch(64, 64, seed=1, teacher=False), dev)
    run = (lambda: model(**b)) if "--eager" in sys.argv else SynthGraphs(model)
    fn = (lambda: run()) if "--eager" in sys.argv else (lambda: run(**b))
    with torch.no_grad():
        for _ in range(3):
            out = fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            out = fn()
        torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call, T_out {out[0].shape[1]}, frames {int(out[9].sum())}")


if __name__ == "__main__":
    main()
