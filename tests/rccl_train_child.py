"""Child process of tests/test_gpu_train.py::test_ddp_step_over_rccl_equals_plain (a helper, not
collected by pytest): the single-rank "nccl" (RCCL) training runs, in their own process, so the
process group's whole lifecycle — init, DDP buckets, collectives captured in a HIP graph, and
the teardown — is checked without sharing the test runner's process.

Teardown order (the round-3 SIGABRT in destroy_process_group): every TrainStep is closed — its
graph (which captured all-reduces on the communicator) reset, the DDP reducer dropped — and the
device drained BEFORE the process group is destroyed. Prints one JSON line with the results and
TEARDOWN_OK after destroy_process_group returned."""
import gc
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (HERE, REPO, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

DEV = "cuda:0"


def main():
    from _common import configs, oracle_state_dict
    from fs2amd import config as C
    from fs2amd.data import synth_batch, to_device
    from fs2amd.model import FastSpeech2
    from fs2amd.trainer import TrainStep

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", rank=0, world_size=1)
    res = {"backend": dist.get_backend(), "runs": []}
    t = torch.ones(1024, device=DEV)
    dist.all_reduce(t)
    res["allreduce_sum"] = float(t.sum())
    pc, mc, _ = configs()
    tc = C.ESD_TRAIN_CONFIG
    # plain eager; DDP (eager, RCCL bucket all-reduces); graph + explicit RCCL all-reduce of the flat
    # gradient buffer in 4 MB slices captured inside the step's HIP graph
    for ddp, graph in ((False, False), (True, False), (True, True)):
        m = FastSpeech2(pc, mc)
        m.load_state_dict(oracle_state_dict())
        m = m.to(DEV).set_precision("fp32")
        m.train_dropout = False
        with TrainStep(m, pc, mc, tc, device=torch.device(DEV), ddp=ddp, bucket_mb=4, graph=graph, warmup=2) as st:
            is_ddp = isinstance(st.net, torch.nn.parallel.DistributedDataParallel)
            base = synth_batch(4, 8, 20, seed=41, with_mels=True, pe_targets=True)
            losses = [float(st(to_device(dict(base, mels=base["mels"] * (1 + 0.1 * i)), DEV))[0]) for i in range(5)]
            torch.cuda.synchronize()
            captured = st._graph is not None
            nbuckets = len(st._buckets) if st.flat else 0
            reduce = st.reduce
        params = {k: p.detach().cpu() for k, p in m.named_parameters()}
        torch.save(params, os.path.join(sys.argv[1], f"params_{len(res['runs'])}.pt"))
        res["runs"].append(dict(ddp=ddp, graph=graph, is_ddp=is_ddp, losses=losses, captured=captured,
                                nbuckets=nbuckets, reduce=reduce))
        del m, st
    gc.collect()
    torch.cuda.synchronize()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    print("TEARDOWN_OK", flush=True)


if __name__ == "__main__":
    main()
