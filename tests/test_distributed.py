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


def _ddp_worker(rank, world, port, q, flat=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.manual_seed(0)
    from _stubs import install_training_stubs
    from _common import configs
    from fs2amd import parallel
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from fs2amd.trainer import TrainStep

    install_training_stubs(setattr)
    r, _, w, dev = parallel.init("gloo")
    pc, mc, tc = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=0)
    m.train_dropout = False
    step = TrainStep(m, pc, mc, tc, device=None, world_size=w, bucket_mb=4, flat_grads=flat)
    assert step.flat == flat
    b = shard(synth_batch(4, 6, 10, seed=9, with_mels=True, pe_targets=True), r, w)
    losses = step(b)
    q.put((r, float(losses[0]), {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}))
    parallel.shutdown()


@pytest.mark.parametrize("flat", [False, True])
def test_ddp_train_step_gloo_world2(monkeypatch, flat):
    """TrainStep over gloo, world 2 (kernels stubbed on CPU, torch ops real): after one step both
    ranks hold identical parameters, equal to one process applying the mean of the two ranks'
    gradients (DDP's all-reduce semantics) with the same ScheduledOptim step. flat=True: the graph
    form's reduction (flat gradient buffer, explicit bucketed all-reduce, 1/world scale, coalesced
    BatchNorm buffer broadcast) run eagerly."""
    from _common import configs
    from _stubs import install_training_stubs
    from fs2amd.data import loss_inputs
    from fs2amd.loss import FastSpeech2Loss
    from fs2amd.model import FastSpeech2
    from fs2amd.optimizer import ScheduledOptim
    from fs2amd.synth_weights import fill_module

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q, flat)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0 = {k: torch.from_numpy(v) for k, v in res[0][2].items()}
    sd1 = {k: torch.from_numpy(v) for k, v in res[1][2].items()}
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k

    # single-process reference: mean of the per-shard gradients, same optimizer step
    install_training_stubs(monkeypatch.setattr)
    pc, mc, tc = configs()
    m = FastSpeech2(pc, mc)
    fill_module(m, seed=0)
    m.train().train_dropout = False
    full = synth_batch(4, 6, 10, seed=9, with_mels=True, pe_targets=True)
    grads = {}
    for r in range(world):
        b = shard(full, r, world)
        m.zero_grad()
        out = m(**b)
        FastSpeech2Loss(pc, mc)(loss_inputs(b), out)[0].backward()
        for k, p in m.named_parameters():
            if p.grad is not None:
                grads[k] = grads.get(k, 0) + p.grad / world
    for k, p in m.named_parameters():
        p.grad = grads.get(k)
    torch.nn.utils.clip_grad_norm_(m.parameters(), tc["optimizer"]["grad_clip_thresh"])
    opt = ScheduledOptim(m, tc, mc, 0)
    opt.step_and_update_lr()
    for k, v in m.state_dict().items():
        if "running_" in k or "num_batches" in k:
            continue  # BN buffers: rank 0's batch statistics (broadcast_buffers)
        torch.testing.assert_close(sd0[k], v, rtol=1e-5, atol=1e-7, msg=k)


def test_bench_launcher_starts_n_ranks():
    """`python bench.py --gpus 2` run as ONE process (the driver's invocation) must start two
    ranks itself and report n_gpus 2 (selftest mode: the same launcher, process group, barrier
    and MAX/SUM bookkeeping as the GPU bench, over gloo)."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--mode", "selftest"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["frames_total"] == 1000 + 2000  # SUM over both ranks
    assert rec["ms_per_step"] >= 20.0 - 1e-6  # MAX over ranks (rank 1 sleeps 20 ms)


def test_flat_grads_accumulation_matches_eager(monkeypatch):
    """grad_acc_step = 2 on the flat-gradient path (the one graph=True / flat_grads=True take) has
    train.py:89-97's semantics: loss / grad_acc_step accumulated over two batches, one clip + Noam
    step every second call. Same parameters as the eager step after 4 calls (2 optimizer steps);
    close() detaches the gradients and refuses further steps."""
    import copy

    from _common import configs
    from _stubs import install_training_stubs
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module
    from fs2amd.trainer import TrainStep

    install_training_stubs(monkeypatch.setattr)
    pc, mc, tc = configs()
    tc = copy.deepcopy(tc)
    tc["optimizer"]["grad_acc_step"] = 2
    sds = []
    for flat in (False, True):
        torch.manual_seed(0)
        m = FastSpeech2(pc, mc)
        fill_module(m, seed=0)
        m.train_dropout = False
        st = TrainStep(m, pc, mc, tc, device=None, flat_grads=flat)
        assert st.flat == flat
        for i in range(4):
            b = synth_batch(3, 6, 10, seed=20 + i, with_mels=True, pe_targets=True)
            st(b)
        assert st.optimizer.current_step == 2
        sds.append({k: v.detach().clone() for k, v in m.state_dict().items()})
        st.close()
        if flat:
            assert all(p.grad is None for p in m.parameters())
            with pytest.raises(RuntimeError):
                st(b)
    for k in sds[0]:
        torch.testing.assert_close(sds[1][k], sds[0][k], rtol=1e-6, atol=1e-8, msg=k)
