"""Interleaved A/B of the NT GEMM's bf16 epilogue in ONE process: dwordx4
stores after a permlane16 swap (default) vs the dwordx2 row-per-lane stores
(MTTS_GEMM_NARROW_OUT=1), on the C2 forward / data-gradient shapes, with
torch (hipBLASLt) alongside.  python tools/gemm_epi_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402

M = 8 * 2048
shapes = {"in_proj": (M, 4096, 1024), "out_proj": (M, 1024, 2048), "q_proj": (M, 1024, 1024),
          "ff1": (M, 2048, 1024), "ff2": (M, 1024, 2048), "dg_in": (M, 1024, 4096), "dg_ff1": (M, 1024, 2048)}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


def timed(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


for name, (m, n, k) in shapes.items():
    a, b = rnd(m, k), rnd(n, k)
    ref = a.float() @ b.float().t()
    res = {"x4": [], "x2": [], "torch": []}
    for _ in range(rounds):
        for arm in res:
            if arm == "x2":
                os.environ["MTTS_GEMM_NARROW_OUT"] = "1"
            else:
                os.environ.pop("MTTS_GEMM_NARROW_OUT", None)
            fn = (lambda: a @ b.t()) if arm == "torch" else (lambda: G.mm_nt(a, b))
            res[arm].append(timed(fn))
    os.environ.pop("MTTS_GEMM_NARROW_OUT", None)
    err = ((G.mm_nt(a, b).float() - ref).abs().max() / ref.abs().max()).item()
    fl = 2 * m * n * k
    line = f"{name:9s} {m}x{n}x{k} err {err:.1e}"
    for arm, v in res.items():
        v.sort()
        line += f"  {arm} {v[len(v) // 2] * 1e3:7.1f}us {fl / v[len(v) // 2] / 1e9:5.0f}TF"
    print(line, flush=True)
