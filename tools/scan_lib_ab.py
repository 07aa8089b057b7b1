"""Per-kernel timing of the selective scan for whichever libmtts.so MTTS_LIB
points at (interleave processes with two libraries for a same-box A/B):
north-star forward (B=32, L=8192, d_inner=2048; fp32 and bf16 I/O) and C2's
forward / backward (B=8, L=2048, d_inner=2048, bf16 I/O, bf16 B/C as the
decoder passes them).  One JSON line: median ms over rounds of HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_ROOT: another package tree (e.g. tools/ab/base: the previous commit's
# Python + library) for a same-box A/B against this tree
PKG = os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from mtts import ops  # noqa: E402


def args(B, L, D, dtype, bc_dtype, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    u = torch.randn(B, L, D, device="cuda", generator=g).to(dtype)
    z = torch.randn(B, L, D, device="cuda", generator=g).to(dtype)
    dl = (torch.randn(B, L, D, device="cuda", generator=g) * 0.1).to(dtype)
    Bm = torch.randn(B, L, 16, device="cuda", generator=g).to(bc_dtype)
    Cm = torch.randn(B, L, 16, device="cuda", generator=g).to(bc_dtype)
    A = -torch.arange(1, 17, device="cuda", dtype=torch.float32).repeat(D, 1)
    Dp = torch.ones(D, device="cuda")
    bias = torch.full((D,), -4.0, device="cuda")
    return u, dl, A, Bm, Cm, Dp, z, bias


def timed(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / iters)
    return sorted(res)[len(res) // 2]


out = {"pkg": os.path.relpath(PKG, ROOT)}
from mtts import _lib  # noqa: E402
paths = {"": None}
if hasattr(_lib, "SCAN_C1P"):   # this tree: also the wave-pair forward
    paths["_c1p"] = _lib.SCAN_C1P
for name, dt in (("ns_fp32", torch.float32), ("ns_bf16", torch.bfloat16)):
    a = args(32, 8192, 2048, dt, dt)
    o = torch.empty_like(a[0])
    for suf, path in paths.items():
        if path is None:
            out[name + suf] = timed(lambda: ops.scan_fwd(*a, True, out=o))
        else:
            with _lib.override(scan_path=path):
                out[name + suf] = timed(lambda: ops.scan_fwd(*a, True, out=o))
    del a, o
    torch.cuda.empty_cache()
a = args(8, 2048, 2048, torch.bfloat16, torch.bfloat16)
out["c2_fwd"] = timed(lambda: ops.scan_fwd(*a, True, want_ckpt=True))
_, _, ck = ops.scan_fwd(*a, True, want_ckpt=True)
dout = torch.randn_like(a[0])
out["c2_bwd"] = timed(lambda: ops.scan_bwd(*a, True, None, ck, dout))
# SWEEP="scan_bwd_segs=2,3,4;scan_segs=1,2": C2 fwd / bwd under each override value
for item in filter(None, os.environ.get("SWEEP", "").split(";")):
    key, vals = item.split("=")
    for v in vals.split(","):
        with _lib.override(**{key: int(v)}):
            out[f"c2_fwd_{key}{v}"] = timed(lambda: ops.scan_fwd(*a, True, want_ckpt=True))
            _, _, ck = ops.scan_fwd(*a, True, want_ckpt=True)
            out[f"c2_bwd_{key}{v}"] = timed(lambda: ops.scan_bwd(*a, True, None, ck, dout))
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
