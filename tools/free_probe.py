#!/usr/bin/env python3
"""Free-running cfg2 synthesis (SynthGraphs) repeated, for rocprofv3 kernel traces: the bench's
free_running_cfg2 leg alone, over 8 distinct seeded batches in rotation (as the bench).
--eager: the eager forward instead."""
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
    bs = [to_device(synth_batch(64, 64, seed=1 + 1000 * i, teacher=False), dev) for i in range(8)]
    synth = SynthGraphs(model)
    fn = (lambda b: model(**b)) if "--eager" in sys.argv else (lambda b: synth(**b))
    with torch.no_grad():
        frames = [int(fn(b)[9].sum()) for b in bs]
        torch.cuda.synchronize()
        cap = synth.captures
        t0 = time.perf_counter()
        for i in range(16):
            out = fn(bs[i % 8])
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 16
    print(f"{dt * 1e3:.3f} ms per call, {sum(frames) / 8 / dt / 1e6:.2f} M frames/s, frames {frames}, "
          f"captures {cap} + {synth.captures - cap} timed, speculation hits {synth.spec_hits} misses {synth.spec_misses}")


if __name__ == "__main__":
    main()
