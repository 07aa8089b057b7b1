"""Per-workgroup cost model of the hand-written NT / TN GEMM kernels: time
C[m,n] = A[m,k] B[n,k]^T (NT, bf16 out) and the TN weight gradient at fixed
output sizes while K grows, so the slope is the steady-state cost of a 64-deep
K-tile and the intercept the fixed prologue / epilogue cost of a workgroup.
python tools/gemm_k_sweep.py   (one JSON line per shape)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3   # us


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


res = []
# NT: 256 output tiles (one round of workgroups) and 1024 tiles (four rounds)
for m, n in ((16384, 1024), (16384, 4096)):
    for k in (512, 1024, 2048, 4096, 8192):
        a, b = rnd(m, k), rnd(n, k)
        us = timed(lambda: G.mm_nt(a, b))
        tiles = (m // 256) * (n // 256)
        res.append({"op": "nt", "m": m, "n": n, "k": k, "tiles": tiles, "us": round(us, 2),
                    "tflops": round(2 * m * n * k / us / 1e6, 1)})
        print(json.dumps(res[-1]), flush=True)
        del a, b
# TN weight gradient: output n x k (1024 x 1024 / 4096 x 1024), reduction over M tokens, each split count
for n, k in ((1024, 1024), (4096, 1024), (1024, 2048)):
    for m in (16384,):
        dy, x = rnd(m, n), rnd(m, k)
        out = torch.empty(n, k, device="cuda")
        for s in (1, 2, 4, 8, 16):
            us = timed(lambda: G.mm_tn(dy, x, out, splits=s))
            res.append({"op": "tn", "m_out": n, "n_out": k, "k_red": m, "splits": s,
                        "wgs": (n // 256) * (k // 256) * s, "us": round(us, 2),
                        "tflops": round(2 * m * n * k / us / 1e6, 1)})
            print(json.dumps(res[-1]), flush=True)
        del dy, x, out
