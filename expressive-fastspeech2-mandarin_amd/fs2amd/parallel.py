"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" on CPU).

Inference shards along the batch: utterances are independent, each rank synthesises its own
shard and there is NO collective on the data path. The only collectives are
the bench's bookkeeping: a barrier around the timed region, a MAX of the per-rank elapsed
time and a SUM of the frames produced.
"""
import os

import torch
import torch.distributed as dist


def env_ranks():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def init(backend=None):
    """Initialise the default process group from torchrun's env (no-op at world size 1).
    Returns (rank, local_rank, world, device)."""
    rank, local, world = env_ranks()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        ndev = torch.cuda.device_count()
        if local >= ndev:  # one process per GPU: never stack two ranks on one device
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} visible GPU(s); launch at most {ndev} ranks")
        dev_index = local
        torch.cuda.set_device(dev_index)
        device = torch.device(f"cuda:{dev_index}")
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world)
    return rank, local, world, device


def barrier():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def aggregate(elapsed_s, frames, device):
    """(max elapsed over ranks, total frames over ranks)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(elapsed_s), int(frames)
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    f = torch.tensor([float(frames)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    return float(t.item()), int(f.item())


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
