#!/usr/bin/env python3
"""attn32_kernel analysis builds: `python tools/attn_abl.py build` makes tracelib/libfs2hip_attn_<v>.so
for the ablation masks below (attention.hip ATTN_ABL bits) and a stamp build (ATTN_TRACE);
`python tools/attn_abl.py run` times the cfg2 decoder attention (packed rows) under each library in
a child process, then prints the stamp build's per-phase cycles.

    python tools/attn_abl.py build && FS2_LIB_ALLOW_MISSING=1 python tools/attn_abl.py run"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "expressive-fastspeech2-mandarin_amd"))
sys.path.insert(0, REPO)
VARIANTS = {"base": 0, "noexp": 1, "noqk": 2, "nopv": 4, "nowait": 8, "nodma": 16, "nomfma": 6, "nomfma_noexp": 7,
            "nodma_noexp": 17}
TL = os.path.join(REPO, "tracelib")


def build():
    """attention.hip per variant, linked with the other objects of the development object cache
    (FS2_OBJ_CACHE, default /tmp/fs2obj: `FS2_OBJ_CACHE=/tmp/fs2obj python __graft_entry__.py` first)."""
    import __graft_entry__ as g
    from fs2amd._lib import source_build_id

    os.makedirs(TL, exist_ok=True)
    cache = os.environ.get("FS2_OBJ_CACHE", "/tmp/fs2obj")
    bid = source_build_id(g.CSRC, os.path.join(REPO, "include", "fs2hip.h"))
    others = [os.path.join(cache, s.replace(".hip", ".o")) for s in g.HIP_SOURCES if s != "attention.hip"]
    flags = {k: [f"-DATTN_ABL={v}"] for k, v in VARIANTS.items()}
    flags["trace"] = ["-DATTN_TRACE=1"]
    procs = {}
    for k, fl in flags.items():
        obj = os.path.join(TL, f"attention_{k}.o")
        procs[k] = (obj, subprocess.Popen(
            ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             f"-I{os.path.join(REPO, 'include')}", f"-I{g.CSRC}", f'-DFS2_BUILD_ID="{bid}"',
             *g.SRC_FLAGS["attention.hip"], *fl, "-c", os.path.join(g.CSRC, "attention.hip"), "-o", obj]))
    for k, (obj, p) in procs.items():
        if p.wait() != 0:
            raise SystemExit(f"attention.hip ({k}) failed")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(TL, f"libfs2hip_attn_{k}.so"), obj, *others], check=True)
        os.remove(obj)


def child(trace):
    import torch
    import bench
    from fs2amd import ops
    from fs2amd.data import synth_batch, to_device

    dev = torch.device("cuda:0")
    model, _, _ = bench.build_model(dev, "bf16")
    bc = synth_batch(64, 64, seed=1)
    b = to_device(bc, dev)
    T = int(bc["max_mel_len"])
    lay = ops.SeqLayout(b["mel_lens"], T)
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(64 * T, 768, generator=g).to(dev, torch.bfloat16)
    fn = lambda: ops.attention(qkv, None, 2, 128, 128 ** 0.5, layout=lay)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"us {e0.elapsed_time(e1) * 1000 / 50:.2f}")
    if trace:
        from fs2amd import _lib
        import numpy as np
        fn()
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 8, dtype=np.uint64)
        _lib.load().fs2_attn_trace_read(ctypes.c_void_p(buf.ctypes.data))
        t = buf.reshape(4096, 8).astype(np.float64)
        t = t[t[:, 6] == 1]
        t0 = t[:, 0].min()
        print(f"workgroups {len(t)}; start skew {t[:, 0].max() - t0:.0f}; span {t[:, 3].max() - t0:.0f} cycles")
        for nt in sorted(set(t[:, 4].astype(int))):
            u = t[t[:, 4] == nt]
            pro, loop, epi = u[:, 1] - u[:, 0], u[:, 2] - u[:, 1], u[:, 3] - u[:, 2]
            print(f"  ntiles {nt:2d} x{len(u):4d}: tiles 0-1 {pro.mean():7.0f} (max {pro.max():7.0f})  "
                  f"rest {loop.mean():7.0f} ({loop.mean() / max(nt - 2, 1):6.0f}/tile)  epilogue {epi.mean():6.0f}  "
                  f"end-to-end {(u[:, 3] - u[:, 0]).mean():7.0f} (max {(u[:, 3] - u[:, 0]).max():7.0f})")
        ends = t[:, 3] - t0
        print(f"  ends: p50 {np.percentile(ends, 50):.0f} p90 {np.percentile(ends, 90):.0f} max {ends.max():.0f}")


def main():
    if sys.argv[1:2] == ["build"]:
        return build()
    if sys.argv[1:2] == ["child"]:
        return child(sys.argv[2] == "1")
    env = dict(os.environ, FS2_LIB_ALLOW_MISSING="1")
    for k in list(VARIANTS) + ["trace"]:
        env["FS2_LIB"] = os.path.join(TL, f"libfs2hip_attn_{k}.so")
        r = subprocess.run([sys.executable, __file__, "child", "1" if k == "trace" else "0"], env=env,
                           capture_output=True, text=True, timeout=150)
        out = [l for l in r.stdout.splitlines() if l.strip()]
        print(f"{k:14s}", "\n".join(out) if r.returncode == 0 else f"FAILED rc {r.returncode}: {r.stderr[-400:]}", flush=True)
        if r.returncode != 0:
            return 1


if __name__ == "__main__":
    sys.exit(main())
