"""In-process interleaved A/B of the GEMM kernels on the C2 shapes:
ping-pong (MTTS_GEMM_PP=1, default) vs the round-2 kernel (MTTS_GEMM_PP=0) vs
torch/hipBLASLt, fwd / dgrad (NT) and wgrad (TN), with an fp32 check."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402

M = 8 * 2048
d, di, dff = 1024, 2048, 2048
shapes = {"in_proj": (M, 2 * di, d), "out_proj": (M, d, di), "q_proj": (M, d, d), "ff1": (M, dff, d),
          "ff2": (M, d, dff)}


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


def rel(x, ref):
    return ((x.float() - ref).abs().max() / ref.abs().max()).item()


def mode(v):
    os.environ["MTTS_GEMM_PP"] = v


tot = {}
for name, (m, n, k) in shapes.items():
    x, w, dy = rnd(m, k), rnd(n, k), rnd(m, n)
    wt = w.t().contiguous()
    fl = 2 * m * n * k
    out_w = torch.empty(n, k, device="cuda")
    cases = {
        "fwd": (lambda: G.mm_nt(x, w), lambda: x @ w.t(), lambda: x.float() @ w.float().t()),
        "dgrad": (lambda: G.mm_nt(dy, wt), lambda: dy @ wt.t(), lambda: dy.float() @ w.float()),
        "wgrad": (lambda: G.mm_tn(dy, x, out_w), None, lambda: dy.float().t() @ x.float()),
    }
    for cname, (ours, blas, ref) in cases.items():
        r = ref()
        errs = {}
        for v in ("2", "1", "0", "3"):
            mode(v)
            errs[v] = rel(ours(), r)
        res = {"ps": [], "pp": [], "pp1": [], "old": [], "blas": []}
        for _ in range(5):
            mode("2"); res["ps"].append(t(ours))
            mode("1"); res["pp"].append(t(ours))
            mode("3"); res["pp1"].append(t(ours))
            mode("0"); res["old"].append(t(ours))
            if blas is not None:
                res["blas"].append(t(blas))
        mode("2")
        med = {kk: sorted(vv)[len(vv) // 2] for kk, vv in res.items() if vv}
        for kk, vv in med.items():
            tot[(cname, kk)] = tot.get((cname, kk), 0.0) + vv
        print(f"{name:8s} {cname:5s} m={m} n={n} k={k}  " + "  ".join(f"{kk} {fl / vv / 1e9:6.0f} TF/s" for kk, vv in med.items())
              + f"  err {max(errs.values()):.1e}", flush=True)
print({f"{a}/{b}": round(v, 3) for (a, b), v in tot.items()})
