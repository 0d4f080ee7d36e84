#!/usr/bin/env python3
"""Mel-synthesis throughput bench (BASELINE.json metric: mel-frames/sec/GPU, batch-64 synth).

One step = one FastSpeech2.forward (eval, bf16 perf mode) over one batch of 64 synthetic
pinyin utterances of 64 phonemes (durations U{2..10} teacher-forced, so
T_max ~ 430 frames; pitch/energy predicted), inputs resident in HBM, random-init weights of
the ESD-Chinese-Singing-MFA architecture from the counter-based generator.

Multi-GPU: one process per GPU (torchrun), each rank synthesises its OWN batch of 64
(weak scaling; utterances are independent, no collective on the data path). The timed
region is bracketed by a barrier + device sync on both sides; the max over ranks is the
job time; value = all valid mel frames of all ranks / job time.

Also reported:
* roofline — the dominant kernel: the decoder's fused FFN (fs2_ffn: Conv1d k=9 + ReLU + Conv1d
  k=1 + residual + LayerNorm, ~86 % of the FLOPs; the conv-k9 launch pair when the fused kernel
  is off or in fp32 / fp8) timed with HIP events on the stream it launches on; achieved =
  algorithmic FLOPs of one op call (valid frames x (2*256*9*1024 + 2*1024*256), or x 2*256*9*1024
  for the conv-k9 alone) / its mean duration inside real forwards, vs the dense MFMA peak.
  ``traffic`` comes from the committed rocprofv3 PMC pass (profiles/) when present.
* decoder_ops — every op of one decoder FFT block (+ the LengthRegulator gather) at the same
  shape, graph-timed, each with its algorithmic work and roofline fraction (bf16 line).
* cpu_baseline — the oracle (CPU restatement of the reference, fp32 PyTorch) on a bounded
  sample of the same workload, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import tempfile
import time
from types import SimpleNamespace

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

HOP, SR = 256, 22050
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
FP8_PEAK_TFLOPS = 5000.0   # dense e4m3 (block-scaled 16x16x128 form)
F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 warm-up forwards: the replayed forwards speed up over the first ~20-30 steps of a run
    # (1.63 -> 1.48 ms per step: clock / power ramp), so the default times the steady state
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--phonemes", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="fp8 = cfg5: FFN Conv1d pair of every FFT block on e4m3 MFMA, the rest bf16")
    ap.add_argument("--graph", type=int, default=1, help="replay the forward as a captured HIP graph")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--vocoder", type=int, default=1, help="also time the HiFi-GAN generator on the cfg2 mel batch")
    ap.add_argument("--extra", type=int, default=1,
                    help="also time free-running cfg2, cfg4 (B=256) and cfg5 (fp8) as extra keys of the JSON line")
    ap.add_argument("--mode", default="infer", choices=["infer", "train", "selftest"],
                    help="infer: the headline cfg2 forward; train: the cfg3 train.py step (B=16/GPU, DDP); "
                         "selftest: the launcher / process-group / timing bookkeeping only (gloo, no GPU)")
    ap.add_argument("--ddp", type=int, default=0,
                    help="train mode: gradient all-reduce over RCCL even at one rank (world > 1 always reduces)")
    ap.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"],
                    help="process-group backend (default: nccl = RCCL; selftest: gloo)")
    return ap.parse_args()


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv, n):
    """``bench.py --gpus N`` started as ONE process: start N rank processes of this same script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env, one GPU each through LOCAL_RANK) and
    exit with the worst exit code. Runs before anything touches the GPU (the parent never
    initialises HIP; the children are fresh interpreters, not exec'd replacements)."""
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def build_model(device, dtype):
    from fs2amd import config as C
    from fs2amd.model import FastSpeech2
    from fs2amd.synth_weights import fill_module

    side = C.write_side_files(tempfile.mkdtemp(prefix="fs2_bench_"))
    pc, mc, _ = C.synthetic_configs(side)
    model = FastSpeech2(pc, mc)
    fill_module(model, seed=0)
    model = model.to(device).eval().set_precision(dtype)
    return model, pc, mc


_SLEEP_CYCLES_PER_MS = []


def _gpu_busy(ms):
    """Keep the launch stream busy for about `ms` (torch.cuda._sleep, calibrated once with HIP
    events) so that the host enqueues a whole eager forward before the GPU reaches it: HIP events
    around each launch then time the kernel, not the host's launch latency."""
    if not _SLEEP_CYCLES_PER_MS:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000)
        e0.record()
        torch.cuda._sleep(2_000_000)
        e1.record()
        e1.synchronize()
        _SLEEP_CYCLES_PER_MS.append(2_000_000 / max(e0.elapsed_time(e1), 1e-3))
    torch.cuda._sleep(int(ms * _SLEEP_CYCLES_PER_MS[0]))


def forward_timers(model, batch, n_fwd=6):
    """HIP events around every launch of interest (fs2amd.runtime.TIMERS: (start, end, tag) in
    launch order) over n_fwd eager forwards, each forward queued behind ~20 ms of GPU work so that
    the timings are kernel durations. Returns [(tag, seconds)] per forward."""
    from fs2amd import runtime

    # one utterance group: the timed launches have the chip to themselves (with stream groups,
    # concurrent launches share the CUs and per-launch durations stop being kernel speed)
    prev = os.environ.get("FS2_STREAMS")
    os.environ["FS2_STREAMS"] = "1"
    per_fwd = []
    try:
        with torch.no_grad():
            model(**batch)
            for _ in range(n_fwd):
                runtime.TIMERS = []
                _gpu_busy(20.0)
                model(**batch)
                per_fwd.append(runtime.TIMERS)
                runtime.TIMERS = None
        torch.cuda.synchronize()
    finally:
        runtime.TIMERS = None
        if prev is None:
            del os.environ["FS2_STREAMS"]
        else:
            os.environ["FS2_STREAMS"] = prev
    return [[(tag, a.elapsed_time(b) / 1e3) for a, b, tag in tms] for tms in per_fwd]


def time_kernel_in_forward(model, batch, n_fwd=6, fwd=None):
    """Mean duration per tag of the timed launches inside real (eager) forwards (forward_timers).
    Returns {tag: (mean seconds, launches)}: decoder FFN tags "fc+ffn" (the last decoder block),
    "fc+ffn+qkv" (blocks 1..5, which also project the next block's Q|K|V), "ffn", "ffn+qkv",
    "ffn8", "conv9"; the other launches "<stack>:<op>"."""
    fwd = forward_timers(model, batch, n_fwd) if fwd is None else fwd
    by = {}
    for tms in fwd:
        for tag, t in tms:
            by.setdefault(tag, []).append(t)
    return {k: (sum(v) / len(v), len(v)) for k, v in by.items()}


GEMM_OPS = {"qkv", "qkv0", "qkv+attn+fc", "fc", "ffn", "ffn+qkv", "fc+ffn", "fc+ffn+qkv", "conv9", "conv1", "ffn8"}
FFT_GEMM_FLOPS_PER_TOKEN = 2 * (256 * 768 + 256 * 256 + 256 * 9 * 1024 + 1024 * 256)  # 5,767,168


def forward_breakdown(fwd, batch_cpu, peak_tflops):
    """Per-forward sums of the timed launches (us), and the two north-star fractions:
    * fft_gemm — every FFT-block GEMM launch of the forward (Q|K|V, fc + LN, the FFN pair, fused
      or not): SURVEY §8d's 5,767,168 FLOP per valid token per layer (QKV + out proj + conv-k9 +
      conv-k1) over the encoder's valid phonemes x 4 layers and the decoder's valid frames x 6,
      divided by the summed durations of those launches, against the dense MFMA peak;
    * lr_fused — the forward's LengthRegulator launch (fs2_lr_fused[_proj]: scan + packed layout +
      gather + PE, and the first decoder Q|K|V by linearity): bytes it must move (x read once,
      durations, the packed frames written, the layout, the projection's operands) over its
      duration, against 8 TB/s. SURVEY §8d's LR quantity itself is lr_gather_table()."""
    n = len(fwd)
    tot = {}
    for tms in fwd:
        for tag, t in tms:
            tot[tag] = tot.get(tag, 0.0) + t / n
    op = lambda tag: tag.split(":", 1)[-1]
    gemm_s = sum(t for tag, t in tot.items() if op(tag) in GEMM_OPS and not tag.startswith("va:"))
    n_gemm = sum(1 for tag, _ in fwd[0] if op(tag) in GEMM_OPS and not tag.startswith("va:"))
    enc_tok = int(batch_cpu["src_lens"].sum())
    frames = int(batch_cpu["mel_lens"].sum()) if batch_cpu.get("mel_lens") is not None else None
    B, Lp = batch_cpu["texts"].shape
    out = {"us_per_forward": {k: round(v * 1e6, 2) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])},
           "forwards_timed": n,
           "timing": "HIP events around each launch on its stream in eager forwards queued behind ~20 ms of GPU "
                     "work (torch.cuda._sleep), so the events bracket the kernel, not the host's launch latency"}
    if frames is not None and gemm_s > 0:
        fl = float(FFT_GEMM_FLOPS_PER_TOKEN) * (4 * enc_tok + 6 * frames)
        if "dec:qkv0" in tot:
            # the decoder's first Q|K|V runs on the phoneme rows (fs2_lr_fused_proj adds the PE term
            # while it gathers): count the FLOPs that GEMM performs, not the frame-level ones
            fl += 2.0 * 256 * 768 * (enc_tok - frames)
        out["fft_gemm"] = {"flops_per_forward": fl, "us_per_forward": round(gemm_s * 1e6, 2), "launches": n_gemm,
                           "achieved": round(fl / gemm_s / 1e12, 2), "peak": peak_tflops, "unit": "TFLOP/s",
                           "frac": round(fl / gemm_s / 1e12 / peak_tflops, 4)}
    lr = tot.get("va:lr")
    if lr and frames is not None:  # the forward's LR launch (with the projection when it carries it)
        T = int(batch_cpu["max_mel_len"])
        byt = B * Lp * 256 * 2.0 + B * Lp * 8.0 + frames * 256 * 2.0 + B * T * 4.0 + frames * 8.0 + (B + 1) * 4.0
        proj = "dec:qkv0" in tot
        if proj:  # fs2_lr_fused_proj: f32 phoneme projection + f32 PE table read once, bf16 Q|K|V written
            byt += B * Lp * 768 * 4.0 + T * 768 * 4.0 + frames * 768 * 2.0
        out["lr_fused"] = {"bytes": byt, "us": round(lr * 1e6, 2), "achieved": round(byt / lr / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(byt / lr / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_note": "bf16 x read once + int64 durations + packed bf16 frames written + rowmap "
                                   "(B*T int32) + row_pos (frames x 8 B) + cu" +
                                   (" + f32 [B*L, 768] phoneme Q|K|V and f32 [T, 768] PE table read once + packed "
                                    "bf16 Q|K|V frames written" if proj else "")}
    return out


def ffn_fused(model, batch, device):
    """Does the benched forward run the decoder FFN as the fused fs2_ffn launch?"""
    from fs2amd import ops, runtime

    P = model.packed(device)
    lp = P.dec_layers[0]
    B, T = batch["d_targets"].shape[0], int(batch["max_mel_len"])
    lay = SimpleNamespace(capacity=B * T) if runtime.packed_decoder_ok(P) else None
    probe = torch.empty(B, T, 0, dtype=ops.torch_dtype(P.act_dtype))
    return lp.fp8 is None and runtime.ffn_fused_ok(P, lp, probe, lay)


def ffn_pre(model, batch, device):
    """Does the benched forward fold the decoder's fc + residual + LN into the fused FFN launch?"""
    from fs2amd import ops, runtime

    P = model.packed(device)
    lp = P.dec_layers[0]
    B, T = batch["d_targets"].shape[0], int(batch["max_mel_len"])
    if not (ffn_fused(model, batch, device) and runtime.packed_decoder_ok(P) and runtime.ffn_pre_on()
            and getattr(lp, "wfcf", None) is not None):
        return False
    probe = torch.empty(B * T, 0)
    return ops.ffn_pre_ok(probe, SimpleNamespace(capacity=B * T), lp.b1.numel(), lp.k1)


def time_dominant_kernel(model, batch, device, reps):
    """Mean duration of the decoder's dominant op (fused FFN, or the FFN conv-k9) run standalone on
    random data; returns (seconds, algorithmic FLOPs per call)."""
    from fs2amd import _lib as L
    from fs2amd import ops

    from fs2amd import runtime

    P = model.packed(device)
    lp = P.dec_layers[0]
    B, T = batch["d_targets"].shape[0], int(batch["max_mel_len"])
    g = torch.Generator(device="cpu").manual_seed(5)
    # the launch the forward makes: packed valid frames (runtime.packed_decoder_ok) or padded rows
    lay = ops.SeqLayout(batch["mel_lens"].to(device), T) if runtime.packed_decoder_ok(P) else None
    shape = (B * T,) if lay is not None else (B, T)
    if lp.fp8 is not None:  # cfg5: the e4m3 launch the forward makes
        h = (torch.randn(*shape, lp.c1, generator=g) * 0.5).to(device=device, dtype=torch.float8_e4m3fn)
        out = torch.empty(*shape, lp.w1.shape[0], device=device, dtype=torch.float8_e4m3fn)
        run = lambda: ops.conv1d(h, lp.fp8.w1, lp.b1, cin=lp.c1, ks=lp.k1, pad=lp.p1, compute=L.FS2_FP8,
                                 epilogue=L.EPI_BIAS_RELU, out=out, out_dtype=L.FS2_FP8, out_scale=1.0 / lp.fp8.s_f,
                                 col_scale=lp.fp8.cs1, layout=lay)
    elif ffn_fused(model, batch, device):
        h = torch.randn(*shape, lp.c1, generator=g).to(device=device, dtype=ops.torch_dtype(P.act_dtype))
        out = torch.empty_like(h)
        pre = None
        if ffn_pre(model, batch, device):  # the forward's launch: fc + residual + LN in the prologue
            att = torch.randn(*shape, lp.c1, generator=g).to(device=device, dtype=ops.torch_dtype(P.act_dtype))
            pre = (att, lp.wfcf, lp.bfc, lp.ln1)
        run = lambda: ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=lp.k1, pad=lp.p1, ln=lp.ln2, layout=lay, out=out, pre=pre)
    else:
        h = torch.randn(*shape, lp.c1, generator=g).to(device=device, dtype=ops.torch_dtype(P.act_dtype))
        out = torch.empty(*shape, lp.w1.shape[0], device=device, dtype=h.dtype)
        run = lambda: ops.conv1d(h, lp.w1, lp.b1, cin=lp.c1, ks=lp.k1, pad=lp.p1, compute=P.compute,
                                 epilogue=L.EPI_BIAS_RELU, out=out, layout=lay)
    for _ in range(3):
        run()
    stream = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    e1.synchronize()
    mean_s = e0.elapsed_time(e1) / 1e3 / reps
    valid = int(batch["mel_lens"].sum())
    flops = 2.0 * valid * lp.c1 * lp.k1 * lp.w1.shape[0]
    if lp.fp8 is None and ffn_fused(model, batch, device):
        flops += 2.0 * valid * lp.c2 * lp.w2.shape[0]
        if ffn_pre(model, batch, device):
            flops += 2.0 * valid * 256 * 256  # the fc of the prologue (valid rows; halo recompute not counted)
    return mean_s, flops


def _graph_mean_s(fn, device, reps):
    """Mean duration of one fn() when `reps` calls run back to back inside one HIP graph (the way
    the bench's graph-replayed forward issues them: no host gap between launches); HIP events on
    the capture stream, which is the stream the kernels launch on."""
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            g.replay()
        e1.record(s)
        e1.synchronize()
    dt = e0.elapsed_time(e1) / 1e3 / (3 * reps)
    del g
    return dt


def decoder_op_table(model, batch_cpu, device, reps):
    """Every decoder op of one FFT block at the benched cfg2 shape (packed valid frames, as the
    forward runs them), each timed as `reps` back-to-back launches in one HIP graph, with its
    algorithmic work per call and the roofline that bounds it:
      ffn    fused FFN (fs2_ffn): conv9 + ReLU + conv1 + res + LN   2*F*(256*9*1024 + 1024*256)  MFMA
      conv9  FFN Conv1d k=9 256->1024 + ReLU   2*F*256*9*1024 FLOP        MFMA
      conv1  FFN Conv1d k=1 1024->256 + res + LN + mask   2*F*1024*256     MFMA
      fc     attention out proj + res + LN + mask          2*F*256*256     MFMA
      qkv    fused Q|K|V projection   F*256*2 in + F*768*2 out + W bytes    HBM
      attn   SDPA, 2 heads of 128     sum_b 4*len_b^2*128*2 FLOP          MFMA
      lr     LengthRegulator gather + decoder PE   B*L*256*2 + B*L*8 in + F*256*2 out  HBM
      lr_fused  the forward's one-launch LR (scan + layout + gather + PE)  lr + cum + layout  HBM
    (F = valid frames; random bf16 inputs of the forward's shapes). bf16 only (the fp8 / fp32 lines
    report the conv-k9 roofline alone). Back-to-back calls of one op keep the matrix pipe busier than
    the forward does, so the MFMA-heavy conv9 reads ~10 % slower here than inside real forwards."""
    from fs2amd import _lib as L
    from fs2amd import ops
    from fs2amd.data import to_device

    P = model.packed(device)
    b = to_device(batch_cpu, device)
    lp = P.dec_layers[0]
    B, T = b["d_targets"].shape[0], int(batch_cpu["max_mel_len"])
    lens = batch_cpu["mel_lens"].long()
    F = int(lens.sum())
    Lp = int(batch_cpu["texts"].shape[1])
    dt = ops.torch_dtype(P.act_dtype)
    g = torch.Generator().manual_seed(0)
    rnd = lambda *s: torch.randn(*s, generator=g).to(device, dt)
    lay = ops.SeqLayout(b["mel_lens"], T)
    h, o, f, qkv = rnd(B * T, 256), rnd(B * T, 256), rnd(B * T, 1024), rnd(B * T, 768)
    x = rnd(B, Lp, 256)
    cum, ml, _ = ops.lr_durations(b["d_targets"])
    ops_ = {
        "ffn": (lambda: ops.ffn(h, lp.w12, lp.b1, lp.b2, ks=9, pad=4, ln=lp.ln2, layout=lay),
                "mfma", 2.0 * F * (256 * 9 * 1024 + 1024 * 256)),
        "conv9": (lambda: ops.conv1d(h, lp.w1, lp.b1, cin=256, ks=9, pad=4, compute=P.compute,
                                     epilogue=L.EPI_BIAS_RELU, out_dtype=P.act_dtype, layout=lay),
                  "mfma", 2.0 * F * 256 * 9 * 1024),
        "conv1_ln": (lambda: ops.conv1d(f, lp.w2, lp.b2, cin=1024, ks=1, pad=0, compute=P.compute,
                                        epilogue=L.EPI_RES_LN, out_dtype=P.act_dtype, residual=h, ln=lp.ln2,
                                        layout=lay),
                     "mfma", 2.0 * F * 1024 * 256),
        "fc_ln": (lambda: ops.conv1d(o, lp.wfc, lp.bfc, cin=256, ks=1, pad=0, compute=P.compute,
                                     epilogue=L.EPI_RES_LN, out_dtype=P.act_dtype, residual=h, ln=lp.ln1, layout=lay),
                  "mfma", 2.0 * F * 256 * 256),
        "qkv": (lambda: ops.conv1d(h, lp.wqkv, lp.bqkv, cin=256, ks=1, pad=0, compute=P.compute,
                                   epilogue=L.EPI_BIAS, out_dtype=P.act_dtype, layout=lay),
                "hbm", F * 256 * 2.0 + F * 768 * 2.0 + 768 * 256 * 2.0),
        "attn": (lambda: ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay),
                 "mfma", float(sum(4.0 * int(n) ** 2 * 128 * 2 for n in lens))),
        "lr": (lambda: ops.lr_expand(x, cum, ml, T, pe=P.dec_pe, out_dtype=P.act_dtype, out_layout=lay),
               "hbm", B * Lp * 256 * 2.0 + B * Lp * 8.0 + F * 256 * 2.0),
        # the forward's LengthRegulator launch (fs2_lr_fused): duration scan + packed layout + gather
        # + PE; algorithmic bytes as "lr" plus the layout it writes (cu, rowmap, row_pos)
        "lr_fused": (lambda: ops.lr_fused(x, b["mel_lens"], T, pe=P.dec_pe, out_dtype=P.act_dtype,
                                          dur=b["d_targets"]),
                     "hbm", B * Lp * 256 * 2.0 + B * Lp * 8.0 * 2 + F * 256 * 2.0 + B * T * 4.0 + F * 8.0 + B * 8.0),
    }
    out = {}
    for name, (fn, bound, work) in ops_.items():
        t = _graph_mean_s(fn, device, reps)
        if bound == "mfma":
            ach, peak, unit, wk = work / t / 1e12, BF16_PEAK_TFLOPS, "TFLOP/s", {"flops_per_call": work}
        else:
            ach, peak, unit, wk = work / t / 1e9, HBM_PEAK_GBS, "GB/s", {"bytes_per_call": work}
        out[name] = {"us": round(t * 1e6, 2), "bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": unit,
                     "frac": round(ach / peak, 4), **wk}
    return out


def lr_gather_table(model, batch_cpu, device, reps):
    """SURVEY §8d's LengthRegulator at the batch's shape, each form timed as `reps` back-to-back
    launches in one HIP graph, random bf16 phoneme rows, the batch's teacher-forced durations:
      padded  fs2_length_regulate, the reference's LengthRegulator.forward + pad contract
              (modules.py:161-194, tools.py:360-378) in one launch: bytes = B*L*D*2 (x read once) +
              B*L*8 (durations) + B*T*D*2 (frames written, zero padding included) + B*8 (mel_len) --
              §8d's formula (cfg2 16.22 MB, cfg4 152.24 MB); its frac is lr_hbm_frac on the line;
      packed  fs2_lr_fused, the forward's form without the Q|K|V projection: scan + packed layout +
              gather + decoder PE into the valid frames only: x + durations + F*D*2 + mel_len + the
              layout (rowmap B*T*4, row_pos F*8, cu) + the f32 PE rows read once (T*D*4)."""
    from fs2amd import ops
    from fs2amd.data import to_device

    P = model.packed(device)
    b = to_device(batch_cpu, device)
    B, Lp = (int(v) for v in batch_cpu["texts"].shape)
    T = int(batch_cpu["max_mel_len"])
    F = int(batch_cpu["mel_lens"].sum())
    D = 256
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, Lp, D, generator=g).to(device, torch.bfloat16)
    dur = b["d_targets"]
    forms = {
        "padded": (lambda: ops.length_regulate(x, dur, T),
                   B * Lp * D * 2.0 + B * Lp * 8.0 + B * T * D * 2.0 + B * 8.0),
        "packed": (lambda: ops.lr_fused(x, b["mel_lens"], T, pe=P.dec_pe, out_dtype=P.act_dtype, dur=dur),
                   B * Lp * D * 2.0 + B * Lp * 8.0 + F * D * 2.0 + B * 8.0 + B * T * 4.0 + F * 8.0 + (B + 1) * 4.0
                   + T * D * 4.0),
    }
    out = {}
    for name, (fn, byt) in forms.items():
        t = _graph_mean_s(fn, device, reps)
        out[name] = {"us": round(t * 1e6, 2), "bytes": byt, "achieved": round(byt / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(byt / t / 1e9 / HBM_PEAK_GBS, 4)}
    out["shape"] = {"B": B, "L": Lp, "T": T, "frames": F}
    return out


def cpu_baseline(batch_cpu, pc, mc, budget_s=20.0):
    """The oracle (reference restatement, fp32 PyTorch CPU, bit-exact to the reference's goldens)
    on the SAME 64-utterance batch the GPU headline runs, repeated for about budget_s seconds."""
    from oracle import fs2_oracle as O
    from fs2amd.synth_weights import synth_state_dict
    from fs2amd import config as C
    from fs2amd.model import FastSpeech2

    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    shapes = {k: tuple(v.shape) for k, v in FastSpeech2(pc, mc).state_dict().items()}
    sd = O.build_state_dict(mc, pc, C.SYNTH_STATS, synth_state_dict(shapes, seed=0))
    frames = int(batch_cpu["mel_lens"].sum())
    with torch.no_grad():
        t0 = time.perf_counter()
        O.forward(sd, mc, pc, **batch_cpu)  # warm-up (also sizes the sample)
        one = time.perf_counter() - t0
        reps = max(1, min(20, int(budget_s / max(one, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            O.forward(sd, mc, pc, **batch_cpu)
        dt = time.perf_counter() - t0
    # single-thread figure on the first 8 utterances of the same batch (one forward, ~5-10 s)
    from fs2amd.data import shard

    sub = shard(batch_cpu, 0, max(1, int(batch_cpu["texts"].shape[0]) // 8))
    sub_frames = int(sub["mel_lens"].sum())
    torch.set_num_threads(1)
    with torch.no_grad():
        t0 = time.perf_counter()
        O.forward(sd, mc, pc, **sub)
        dt1 = time.perf_counter() - t0
    torch.set_num_threads(threads)
    B = int(batch_cpu["texts"].shape[0])
    return {"value": round(frames * reps / dt, 1), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "value_1thread": round(sub_frames / dt1, 1),
            "sample": f"oracle fp32 forward on the benched cfg2 batch ({B} utterances, {frames} frames) x {reps} "
                      f"reps after 1 warm-up, {dt:.1f} s, torch.set_num_threads({threads}) (the box's CPU share; "
                      f"os.cpu_count() = {os.cpu_count()} is the whole host); value_1thread: one forward of its "
                      f"first {int(sub['texts'].shape[0])} utterances ({sub_frames} frames) on 1 thread, {dt1:.1f} s"}


def load_traffic(dtype="bf16", fused=False, pre=False):
    name = ("ffn_pre_traffic.json" if pre else "ffn_traffic.json") if fused else \
        ("conv9_traffic.json" if dtype == "bf16" else f"conv9_{dtype}_traffic.json")
    path = os.path.join(REPO, "profiles", name)
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    return None


def train_workload(args, rank, world, device, steps, warmup, ddp=False):
    """cfg3: one train.py step per iteration (forward, FastSpeech2Loss, backward, RCCL gradient
    all-reduce, clip, ScheduledOptim) on B=16 utterances per GPU, lengths U{16..64}, mel / pitch
    / energy targets N(0,1), timed as the headline is (barrier + device sync on both sides, max over
    ranks). value = mel frames of all ranks per second. Returns the record (fields of a bench line)."""
    from fs2amd import config as C
    from fs2amd import parallel
    from fs2amd.data import synth_batch, to_device
    from fs2amd.trainer import TrainStep

    model, pc, mc = build_model(device, args.dtype)
    _, _, tc = C.synthetic_configs(tempfile.mkdtemp(prefix="fs2_bench_tc_"))
    B = 16
    batch_cpu = synth_batch(B, 16, 64, seed=1 + rank, with_mels=True, pe_targets=True)
    batch = to_device(batch_cpu, device)
    frames = int(batch_cpu["mel_lens"].sum())
    if ddp and world == 1 and not torch.distributed.is_initialized():
        # a single-rank RCCL group, so the step's all-reduce path runs (and is timed) on one GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        torch.distributed.init_process_group("nccl", init_method="env://", rank=0, world_size=1)
    step = TrainStep(model, pc, mc, tc, device=device, world_size=world, graph=bool(args.graph),
                     ddp=ddp or world > 1)
    try:
        for _ in range(max(1, warmup)):
            step(batch)
        torch.cuda.synchronize(device)
        parallel.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(steps):
            losses = step(batch)
        torch.cuda.synchronize(device)
        parallel.barrier()
        elapsed = time.perf_counter() - t0
        elapsed, tot_frames = parallel.aggregate(elapsed, frames, device)
        return {
            "metric": "train mel-frames/sec (cfg3 train.py step, batch 16/GPU, DDP over RCCL)",
            "value": round(tot_frames * steps / elapsed, 1), "unit": "mel-frames/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (pinyin ids U{64..107}, lengths U{16..64}, durations U{2..10}, mel/pitch/energy "
                    "targets N(0,1); counter-generated random-init weights)",
            "config": {"workload": "cfg3: FastSpeech2 train step, ESD-Chinese-Singing-MFA model.yaml",
                       "global_batch": B * world, "frames_per_gpu_batch": frames,
                       "parallelism": (f"dp{world} (flat fp32 gradient buffer all-reduced over RCCL in 32 MB "
                                       "slices inside the step's HIP graph)" if step.graph_mode and step.reduce else
                                       f"dp{world} (DDP over RCCL, 32 MB buckets)" if step.reduce else
                                       "dp1 (one GPU, no collective)"),
                       "hip_graph": step.graph_mode},
            "loss": round(float(losses[0]), 5),
        }
    finally:
        # the graph holds the captured RCCL all-reduces: release it (device drained) before the
        # communicator is destroyed
        step.close()


def main_train(args, rank, world, device):
    """``--mode train``: the cfg3 step (train_workload) as the bench line."""
    from fs2amd import parallel

    rec = train_workload(args, rank, world, device, args.steps, args.warmup, ddp=bool(args.ddp))
    if rank == 0:
        print(json.dumps(rec), flush=True)
    parallel.shutdown()


def timed_steps(model, batch, device, steps, warmup, graph, frames_out=None):
    """W untimed warmups, then EXACTLY `steps` forwards bracketed by barrier + device sync on both
    sides; returns this rank's elapsed seconds. graph: the forward is captured once as a HIP graph
    and replayed (needs a sync-free forward: teacher-forced / max_mel_len given)."""
    from fs2amd import parallel

    def step():
        with torch.no_grad():
            return model(**batch)

    for _ in range(max(1, warmup)):
        out = step()
    torch.cuda.synchronize(device)
    run = step
    if graph:
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream(device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # captured on the warm-up stream: its split-K workspace already exists, so the graph holds
        # no counter-zeroing memset (ops.splitk_workspace is per stream)
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            out = step()
        g.replay()
        torch.cuda.synchronize(device)
        run = g.replay
    if frames_out is not None:
        frames_out.append(int(out[9].sum()))
    parallel.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize(device)
    parallel.barrier()
    return time.perf_counter() - t0


def extra_workloads(model, args, rank, device):
    """The other BASELINE configs as extra keys on the same JSON line (same barrier / MAX-over-
    ranks bookkeeping, fewer steps):
    * free_running_cfg2 — the synthesis path of synthesize_chinese_pinyin.py:140-145: durations
      predicted and rounded, no max_mel_len, so one device->host read of max(mel_len) per
      forward and no graph capture (eager launches);
    * cfg4_b256 — B=256, 16..160 phonemes, teacher-forced, graph-replayed (LengthRegulator and
      ragged-padding stress);
    * cfg5_fp8 — cfg2 with the FFN pair (and Q|K|V of blocks 1..n) on e4m3 MFMA, graph-replayed
      (only when the headline runs bf16)."""
    from fs2amd import parallel
    from fs2amd.data import synth_batch, to_device

    res = {}
    steps = max(3, args.steps // 2)
    prec = model.precision

    def record(name, batch_cpu, graph, note):
        b = to_device(batch_cpu, device)
        got = []
        el = timed_steps(model, b, device, steps, 2, graph, frames_out=got)
        el, fr = parallel.aggregate(el, got[0], device)
        res[name] = {"value": round(fr * steps / el, 1), "unit": "mel-frames/s", "ms_per_step": round(el / steps * 1e3, 4),
                     "steps": steps, "frames_per_step": fr, "hip_graph": graph, "dtype": model.precision, "note": note}

    record("free_running_cfg2_eager", synth_batch(args.batch, args.phonemes, seed=1 + rank, teacher=False), False,
           "durations predicted + rounded (modules.py:131-137), one D2H read of max(mel_len), eager launches")
    res["free_running_cfg2"] = synth_graphs_workload(model, args, rank, device, steps)
    b4 = synth_batch(256, 16, 160, seed=1 + rank)
    record("cfg4_b256", b4, True, "B=256 x U{16..160} phonemes, teacher-forced durations U{2..10}")
    # the LengthRegulator stress shape (152 MB bf16): its launch inside eager cfg4
    # forwards, and the FFT-block GEMM fraction at B=256
    pk4 = {"bf16": BF16_PEAK_TFLOPS, "fp8": FP8_PEAK_TFLOPS}.get(prec, F32_PEAK_TFLOPS)
    brk4 = forward_breakdown(forward_timers(model, to_device(b4, device), n_fwd=3), b4, pk4)
    for k in ("lr_fused", "fft_gemm"):
        if k in brk4:
            res["cfg4_b256"][k] = brk4[k]
    if prec == "bf16":
        # SURVEY §8d's LengthRegulator quantity at the stress shape (152 MB bf16)
        res["cfg4_b256"]["lr"] = lr_gather_table(model, b4, device, args.kernel_reps)
        res["cfg4_b256"]["lr_hbm_frac"] = res["cfg4_b256"]["lr"]["padded"]["frac"]
    if prec == "bf16":
        cal = synth_batch(args.batch, args.phonemes, seed=1000 + rank)
        b5 = synth_batch(args.batch, args.phonemes, seed=1 + rank)
        # cfg5's tolerance against bf16 on the benched batch: teacher-forced durations, pitch / energy
        # pinned to the bf16 predictions (no bucket can flip), valid frames (tests/test_gpu_fp8.py)
        with torch.no_grad():
            bd = to_device(b5, device)
            r16 = model(**bd)
            pinned = dict(bd, p_targets=r16[2].clone(), e_targets=r16[3].clone())
            r16 = model(**pinned)
            model.set_precision("fp8")
            model.calibrate_fp8(**to_device(cal, device))
            r8 = model(**pinned)
            valid = (torch.arange(r16[1].shape[1], device=device)[None, :] < r16[9][:, None])[..., None]
            err = (r8[1].float() - r16[1].float()).abs().masked_select(valid)
            tol = {"postnet_max_abs": round(float(err.max()), 5), "postnet_mean_abs": round(float(err.mean()), 6),
                   "reference": "bf16 forward, same batch, pitch / energy pinned to its predictions, valid frames",
                   "asserted": "tests/test_gpu_fp8.py::test_fp8_model_vs_bf16_reported"}
        record("cfg5_fp8", b5, True, "cfg2 with e4m3 FFN + Q|K|V GEMMs (static calibrated scales)")
        res["cfg5_fp8"]["tol_vs_bf16"] = tol
        # the fused e4m3 FFN (fs2_ffn8) against the dense fp8 peak: HIP events around its launches in
        # eager forwards (all 6 decoder blocks)
        t8 = time_kernel_in_forward(model, to_device(b5, device))
        if "ffn8" in t8:
            s8, n8 = t8["ffn8"]
            fl8 = 2.0 * int(b5["mel_lens"].sum()) * (256 * 9 * 1024 + 1024 * 256)
            res["cfg5_fp8"]["roofline"] = {
                "bound": "mfma", "kernel": "ffn8_fused_kernel (decoder FFN, e4m3 v_mfma_scale_f32_16x16x128_f8f6f4)",
                "achieved": round(fl8 / s8 / 1e12, 2), "peak": FP8_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(fl8 / s8 / 1e12 / FP8_PEAK_TFLOPS, 4), "kernel_ms": round(s8 * 1e3, 4),
                "launches_timed": n8, "flops_per_launch": fl8}
        model.set_precision(prec)
    if args.vocoder:
        res["vocoder_cfg2"] = vocoder_workload(model, args, rank, device, steps)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and prec in ("bf16", "fp32"):
        # cfg3 on the driver's record: one graphed TrainStep at B=16 (the --mode train line's step);
        # one GPU only (at N > 1 this line stays the inference bench: the in-graph RCCL all-reduce
        # is exercised by `bench.py --mode train`, not inside the scaling runs)
        tr = train_workload(SimpleNamespace(dtype=prec, graph=1), rank, world, device, max(20, steps), 5)
        res["train_cfg3"] = {k: tr[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "loss")}
        res["train_cfg3"].update(frames_per_step=tr["config"]["frames_per_gpu_batch"],
                                 hip_graph=tr["config"]["hip_graph"], parallelism=tr["config"]["parallelism"],
                                 note="cfg3 train.py step (forward, FastSpeech2Loss, backward, clip_grad_norm_, "
                                      "ScheduledOptim Adam) on B=16 x U{16..64} phonemes, one HIP graph per step")
    return res


def synth_graphs_workload(model, args, rank, device, steps, n_batches=8):
    """The synthesis path (free-running cfg2: predicted durations, no max_mel_len) as a serving
    loop runs it: ``n_batches`` DISTINCT seeded batches of 64 x 64 phonemes called in rotation, each
    timed call a whole synthesis call including its one host read. Through
    fs2amd.graphs.SynthGraphs (stage-1 graph, the host read, the decoder graph of the T bucket, the
    eager T_out-shaped tail) and, for comparison, the eager forward on the same rotation. One
    warm-up pass over the batches captures what it needs; the captures of the timed calls are
    counted (a serving loop must not recapture per batch)."""
    from fs2amd import parallel
    from fs2amd.data import synth_batch, to_device
    from fs2amd.graphs import SynthGraphs

    bs = [to_device(synth_batch(args.batch, args.phonemes, seed=1 + rank + 1000 * i, teacher=False), device)
          for i in range(n_batches)]
    synth = SynthGraphs(model)
    res = {}
    for name, fn in (("graphs", lambda b: synth(**b)), ("eager", lambda b: model(**b))):
        frames, t_out = [], []
        with torch.no_grad():
            for b in bs:
                out = fn(b)
                frames.append(int(out[9].sum()))
                t_out.append(int(out[0].shape[1]))
        torch.cuda.synchronize(device)
        cap0 = synth.captures
        parallel.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        with torch.no_grad():
            for i in range(steps):
                fn(bs[i % n_batches])
        torch.cuda.synchronize(device)
        parallel.barrier()
        fr = sum(frames[i % n_batches] for i in range(steps))
        el, fr = parallel.aggregate(time.perf_counter() - t0, fr, device)
        res[name] = {"value": round(fr / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
                     "frames_per_step_mean": round(fr / steps, 1), "T_out": t_out,
                     **({"graphs_captured_warmup": cap0, "graphs_captured_timed": synth.captures - cap0,
                         "speculation_hits": synth.spec_hits, "speculation_misses": synth.spec_misses}
                        if name == "graphs" else {})}
    synth.close()
    g = res["graphs"]
    return {"value": g["value"], "unit": "mel-frames/s", "ms_per_step": g["ms_per_step"], "steps": steps,
            "distinct_batches": n_batches, "frames_per_step_mean": g["frames_per_step_mean"], "T_out": g["T_out"],
            "hip_graph": True, "dtype": model.precision,
            "graphs_captured_warmup": g["graphs_captured_warmup"], "graphs_captured_timed": g["graphs_captured_timed"],
            "speculation": {"hits": g["speculation_hits"], "misses": g["speculation_misses"]},
            "eager": {k: res["eager"][k] for k in ("value", "ms_per_step")},
            "note": "durations predicted + rounded (modules.py:131-137); 8 distinct seeded batches in rotation; "
                    "fs2amd.graphs.SynthGraphs: stage-1 graph, ONE device->host read (max / sum of mel_len + "
                    "bad-id count) with the decoder graph of the recent calls' buckets replayed speculatively "
                    "under it (kept when the call fits them with the same launch forms), the T_out-shaped "
                    "mel_linear / PostNet tail issued eagerly behind it; 'eager': the eager forward on the "
                    "same rotation"}


def vocoder_workload(model, args, rank, device, steps):
    """HiFi-GAN V1 (hifigan/models.py, random-init weights) on the cfg2 batch's postnet mel
    [64, T_max, 80] (padded, as synth_samples hands it over), graph-replayed, same precision as
    the headline; plus the end-to-end synthesis rate (acoustic model + vocoder, both replayed)."""
    from fs2amd import parallel
    from fs2amd.data import synth_batch, to_device
    from fs2amd.synth_weights import fill_vocoder
    from fs2amd.vocoder import V1_CONFIG, Generator, flops_per_frame

    voc = Generator(V1_CONFIG)
    fill_vocoder(voc, V1_CONFIG, seed=0)
    voc = voc.to(device).eval()
    voc.remove_weight_norm()
    voc.set_precision("bf16" if model.precision in ("bf16", "fp8") else "fp32")
    b = to_device(synth_batch(args.batch, args.phonemes, seed=1 + rank), device)
    with torch.no_grad():
        mel = model(**b)[1]
    frames_valid = int(b["mel_lens"].sum())
    B, T, _ = mel.shape

    def step():
        with torch.no_grad():
            return voc.forward_btc(mel)

    for _ in range(2):
        step()
    torch.cuda.synchronize(device)
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        step()
    g.replay()
    torch.cuda.synchronize(device)
    parallel.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize(device)
    parallel.barrier()
    el, fr = parallel.aggregate(time.perf_counter() - t0, frames_valid, device)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    ms = el / steps * 1e3
    tflops = flops_per_frame() * B * T / (el / steps) / 1e12
    return {"value": round(fr * steps / el, 1), "unit": "mel-frames/s (valid frames vocoded)", "ms_per_step": round(ms, 3),
            "steps": steps, "frames_per_step_padded": B * T, "samples_per_step": B * T * voc.hop,
            "dtype": voc._precision, "achieved_tflops": round(tflops, 1),
            "flops_per_frame": flops_per_frame(), "hip_graph": True,
            "rtf_vocoder": round((el / steps) / (fr / world * HOP / SR), 7),
            "note": "HiFi-GAN V1 on the padded cfg2 postnet mel (synth_samples / vocoder_infer input); "
                    "FLOPs counted on the padded frames it computes"}


def main_selftest(args, rank, world, device):
    """The N-rank bookkeeping of the bench without a model: barrier + timed region + MAX/SUM over
    ranks, one JSON line from rank 0 (tests/test_distributed.py runs it over gloo on CPU)."""
    from fs2amd import parallel

    frames = 1000 * (rank + 1)
    parallel.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    parallel.barrier()
    elapsed, tot = parallel.aggregate(time.perf_counter() - t0, frames, device)
    if rank == 0:
        print(json.dumps({"metric": "bench launcher self-test", "value": round(tot / elapsed, 1), "unit": "frames/s",
                          "n_gpus": world, "steps": 1, "warmup": 0, "ms_per_step": round(elapsed * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "none",
                          "data": "none", "config": {"workload": "selftest", "frames_total": tot,
                                                     "backend": device.type}}), flush=True)
    parallel.shutdown()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's single-process `bench.py --gpus N`: become the launcher of N ranks
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    from fs2amd import parallel

    backend = args.backend or ("gloo" if args.mode == "selftest" else "nccl")
    rank, local, world, device = parallel.init(backend)
    if world != args.gpus and rank == 0:
        print(f"bench: note: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the {world} ranks that ran",
              file=sys.stderr, flush=True)
    if args.mode == "selftest":
        return main_selftest(args, rank, world, device)
    if args.mode == "train":
        return main_train(args, rank, world, device)

    from fs2amd.data import synth_batch, to_device

    model, pc, mc = build_model(device, args.dtype)
    batch_cpu = synth_batch(args.batch, args.phonemes, seed=1 + rank)
    batch = to_device(batch_cpu, device)
    frames = int(batch_cpu["mel_lens"].sum())

    if args.dtype == "fp8":
        # static activation scales from a calibration batch of the same shape (different seed)
        model.calibrate_fp8(**to_device(synth_batch(args.batch, args.phonemes, seed=1000 + rank), device))

    elapsed = timed_steps(model, batch, device, args.steps, args.warmup, bool(args.graph))
    elapsed, tot_frames = parallel.aggregate(elapsed, frames, device)
    extra = extra_workloads(model, args, rank, device) if args.extra else {}

    fwd_t = forward_timers(model, batch)
    timed = time_kernel_in_forward(model, batch, fwd=fwd_t)
    eager_s, n_launch = timed.get("fc+ffn", timed.get("ffn", timed.get("conv9", (float("nan"), 0))))
    standalone_s, kernel_flops = time_dominant_kernel(model, batch_cpu, device, args.kernel_reps)
    table = None
    if args.dtype == "bf16":
        try:  # diagnostics only: never lose the headline line to them
            table = decoder_op_table(model, batch_cpu, device, args.kernel_reps)
        except Exception as e:  # noqa: BLE001
            print(f"bench: decoder op table failed: {e!r}", file=sys.stderr, flush=True)
    # the op inside real forwards (interleaved with the block's lighter launches, as in the bench);
    # back-to-back calls (decoder_ops) run slower (likely clocks under sustained MFMA load)
    kernel_s = eager_s
    fused = ffn_fused(model, batch_cpu, device)
    pre = fused and ffn_pre(model, batch_cpu, device)
    qtag = "fc+ffn+qkv" if pre else "ffn+qkv"
    timing = ("HIP events around the last decoder block's fused launch (fc + residual + LN, then the FFN) in 6 "
              "eager forwards (blocks 1-5 also project the next block's Q|K|V: 'with_next_qkv')" if pre else
              "HIP events around the last decoder block's fused-FFN launch in 6 eager forwards (blocks 1-5 "
              "also project the next block's Q|K|V: 'with_next_qkv')" if fused else
              "HIP events around each decoder conv-k9 op call (both launches) in 6 eager forwards")
    ms_per_step = elapsed / args.steps * 1e3
    value = tot_frames * args.steps / elapsed
    peak = {"bf16": BF16_PEAK_TFLOPS, "fp8": FP8_PEAK_TFLOPS}.get(args.dtype, F32_PEAK_TFLOPS)
    achieved = kernel_flops / kernel_s / 1e12
    rec = {
        "metric": "mel-frames/sec/GPU (batch-64 synth) at 1/2/4/8 MI355X; RTF",
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "per_gpu": round(value / world, 1),  # value is the whole-job aggregate (all ranks' frames / max time)
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded pinyin ids U{64..107}, durations U{2..10} teacher-forced, pitch/energy "
                "predicted; counter-generated random-init weights)",
        "config": {"workload": f"cfg2: batch={args.batch} x {args.phonemes} phonemes per GPU, ESD-Chinese-Singing-MFA "
                               f"model.yaml, FastSpeech2.forward eval {args.dtype}",
                   "global_batch": args.batch * world, "seq_len": args.phonemes,
                   "mel_frames_per_gpu_batch": frames, "T_max": int(batch_cpu["max_mel_len"]),
                   "parallelism": f"dp{world} (independent shards, no collective)",
                   "hip_graph": bool(args.graph)},
        "rtf": round((elapsed / args.steps) / (tot_frames / world * HOP / SR), 7),
        "roofline": {"bound": "mfma", "kernel": ("decoder FFT block after attention (bf16): ffn_fused_kernel<PRE> = fc "
                                                 "256->256 + residual + LayerNorm, Conv1d k=9 256->1024 + ReLU + "
                                                 "Conv1d k=1 1024->256 + residual + LayerNorm, one launch"
                                                 if pre else
                                                 "decoder FFN fused (bf16): ffn_fused_kernel = Conv1d k=9 256->1024 + "
                                                 "ReLU + Conv1d k=1 1024->256 + residual + LayerNorm, one launch"
                                                 if fused else
                                                 f"decoder FFN Conv1d k=9, 256->1024 ({args.dtype}): "
                                                 + ("conv_gemm_8p_kernel whole rounds + conv_gemm_kernel rows left"
                                                    if args.dtype == "bf16" else "conv_gemm_kernel")),
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": load_traffic(args.dtype, fused, pre),
                     "kernel_ms": round(kernel_s * 1e3, 4), "timing": timing,
                     "op_calls_timed": n_launch,
                     "kernel_ms_standalone_random": round(standalone_s * 1e3, 4),
                     "flops_per_launch": kernel_flops,
                     **({"with_next_qkv": {
                         "kernel_ms": round(timed[qtag][0] * 1e3, 4), "launches": timed[qtag][1],
                         "flops_per_launch": kernel_flops + 2.0 * frames * 256 * 768,
                         "achieved": round((kernel_flops + 2.0 * frames * 256 * 768) / timed[qtag][0] / 1e12, 2)}}
                        if qtag in timed else {}),
                     "traffic_note": "2*FETCH_SIZE + WRITE_SIZE per launch (rocprofv3 PMC, profiles/"
                                     + ("ffn_pre_traffic.json: this launch inside eager cfg2 forwards, round 5)"
                                        if pre else "ffn_traffic.json)" if fused else "conv9_traffic.json)")},
    }
    # the north-star fractions: HIP events around every launch of eager forwards (queued behind GPU
    # work, so they bracket kernels); graph-replayed kernel times are 2-5 % shorter (rocprof traces)
    brk = forward_breakdown(fwd_t, batch_cpu, peak)
    if "fft_gemm" in brk:
        rec["fft_gemm_frac"] = brk["fft_gemm"]["frac"]
    if args.dtype == "bf16":
        # SURVEY §8d's LengthRegulator: scan + gather (+ decoder PE) alone, bytes = x read once +
        # durations + frames written + mel_len; the forward's launch, which also projects the first
        # decoder Q|K|V, is forward_breakdown.lr_fused
        lrt = lr_gather_table(model, batch_cpu, device, args.kernel_reps)
        rec["lr_hbm_frac"] = lrt["padded"]["frac"]
        rec["lr"] = lrt
    rec["forward_breakdown"] = brk
    if table is not None:
        rec["decoder_ops"] = table
    if rank == 0 and world == 1 and args.cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(batch_cpu, pc, mc)
    if extra:
        rec["extra"] = extra
    if rank == 0:
        print(json.dumps(rec), flush=True)
    parallel.shutdown()


if __name__ == "__main__":
    main()
