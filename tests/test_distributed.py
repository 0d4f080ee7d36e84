"""N>1 path on CPU: batch sharding and the bench's rank bookkeeping over gloo (world size 2)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from fs2amd.data import shard, synth_batch


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shards_partition_the_batch(world):
    b = synth_batch(64, 16, 64, seed=3)
    seen = []
    for r in range(world):
        s = shard(b, r, world)
        n = s["texts"].shape[0]
        assert s["max_src_len"] == int(s["src_lens"].max()) == s["texts"].shape[1]
        assert s["max_mel_len"] == int(s["mel_lens"].max())
        assert torch.equal(s["mel_lens"], s["d_targets"].sum(1))
        seen.append(s["texts"][:, :8])
        assert n == 64 // world
    assert torch.equal(torch.cat(seen), b["texts"][:, :8])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from fs2amd import parallel

    r, local, w, dev = parallel.init("gloo")
    parallel.barrier()
    b = shard(synth_batch(8, 12, 20, seed=5), r, w)
    frames = int(b["mel_lens"].sum())
    elapsed = 0.5 + r  # rank-dependent fake time
    e, f = parallel.aggregate(elapsed, frames, dev)
    q.put((r, e, f, frames))
    parallel.shutdown()


def test_gloo_world2_aggregation():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = sum(r[3] for r in res)
    full = int(synth_batch(8, 12, 20, seed=5)["mel_lens"].sum())
    assert total == full
    for r, e, f, _ in res:
        assert e == 1.5 and f == full
