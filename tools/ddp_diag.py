#!/usr/bin/env python3
"""Diagnostics for test_ddp_step_over_rccl_equals_plain: parameter differences after 5 steps for
plain (twice), DDP eager and graph + flat all-reduce, single-rank RCCL group."""
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from _common import configs, oracle_state_dict
    from fs2amd import config as C
    from fs2amd.data import synth_batch, to_device
    from fs2amd.model import FastSpeech2
    from fs2amd.trainer import TrainStep

    DEV = "cuda:0"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", rank=0, world_size=1)
    pc, mc, _ = configs()
    tc = C.ESD_TRAIN_CONFIG
    runs = []
    for ddp, graph in ((False, False), (False, False), (True, False), (True, True), (False, True)):
        m = FastSpeech2(pc, mc)
        m.load_state_dict(oracle_state_dict())
        m = m.to(DEV).set_precision("fp32")
        m.train_dropout = False
        st = TrainStep(m, pc, mc, tc, device=torch.device(DEV), ddp=ddp, bucket_mb=4, graph=graph, warmup=2)
        base = synth_batch(4, 8, 20, seed=41, with_mels=True, pe_targets=True)
        losses = [float(st(to_device(dict(base, mels=base["mels"] * (1 + 0.1 * i)), DEV))[0]) for i in range(5)]
        torch.cuda.synchronize()
        runs.append(((ddp, graph), losses, {k: p.detach().clone() for k, p in m.named_parameters()}))
    tag0, l0, p0 = runs[0]
    lr = st.optimizer._optimizer.param_groups[0]["lr"]
    print("lr", float(lr))
    for tag, l, p in runs[1:]:
        worst = max(((float((p[k] - p0[k]).abs().max()), k) for k in p0))
        nbad = sum(int((~torch.isclose(p[k], p0[k], rtol=1e-4, atol=1e-6)).sum()) for k in p0)
        print(tag, "loss rel", max(abs(a - b) / abs(b) for a, b in zip(l, l0)), "param max diff", worst, "n outside tol", nbad)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
