"""mtts_gemm (hand-written MFMA) vs torch/hipBLASLt on every C2 GEMM shape:
fwd (NT), dgrad (NT on Wᵀ), wgrad (TN, fp32 out), with a correctness check
against an fp32 product of the same bf16 operands.  Uniform [-1, 1) data."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402

M = 8 * 2048
d, di, r, N, dff, S = 1024, 2048, 64, 16, 2048, 8 * 128
shapes = {  # name: (m, n, k) for y[m,n] = x[m,k] W[n,k]^T
    "in_proj": (M, 2 * di, d), "x_proj": (M, r + 2 * N, di), "dt_proj": (M, di, r), "out_proj": (M, d, di),
    "q_proj": (M, d, d), "kv_proj": (S, 2 * d, d), "ff1": (M, dff, d), "ff2": (M, d, dff),
}
only = sys.argv[1].split(",") if len(sys.argv) > 1 else None


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


tot = {"ours": 0.0, "torch": 0.0}
for name, (m, n, k) in shapes.items():
    if only and name not in only:
        continue
    x, w, dy = rnd(m, k), rnd(n, k), rnd(m, n)
    wt = w.t().contiguous()
    fl = 2 * m * n * k
    line = [f"{name:9s} m={m:6d} n={n:5d} k={k:5d}"]
    if G.nt_ok(x, w):
        ref = x.float() @ w.float().t()
        e = rel(G.mm_nt(x, w), ref)
        to, tt = t(lambda: G.mm_nt(x, w)), t(lambda: x @ w.t())
        line.append(f"fwd {fl / to / 1e9:5.0f} vs {fl / tt / 1e9:5.0f} TF/s err {e:.1e}")
        tot["ours"] += to
        tot["torch"] += tt
    if G.nt_ok(dy, wt):
        ref = dy.float() @ w.float()
        e = rel(G.mm_nt(dy, wt), ref)
        to, tt = t(lambda: G.mm_nt(dy, wt)), t(lambda: dy @ wt.t())
        line.append(f"dgrad {fl / to / 1e9:5.0f} vs {fl / tt / 1e9:5.0f} err {e:.1e}")
        tot["ours"] += to
        tot["torch"] += tt
    if G.tn_ok(dy, x):
        ref = dy.float().t() @ x.float()
        out = torch.empty(n, k, device="cuda")
        e = rel(G.mm_tn(dy, x, out), ref)
        res = {}
        for s in (1, 2, 4, 8, 16):
            if m % (64 * s) == 0:
                res[s] = t(lambda: G.mm_tn(dy, x, out, splits=s))
        sb = min(res, key=res.get)
        to = res[G.tn_splits(n, k, m)]
        mm = m // 4
        tt = t(lambda: torch.bmm(dy.view(4, mm, n).transpose(1, 2), x.view(4, mm, k), out_dtype=torch.float32).sum(0))
        line.append(f"wgrad {fl / to / 1e9:5.0f} (s={G.tn_splits(n, k, m)}; best s={sb} {fl / res[sb] / 1e9:5.0f}) "
                    f"vs {fl / tt / 1e9:5.0f} err {e:.1e}")
        tot["ours"] += to
        tot["torch"] += tt
    print("  ".join(line), flush=True)
print(f"total ms: ours {tot['ours']:.3f} torch {tot['torch']:.3f}")

# epilogues (ff1 fwd + bias + gelu; ff2 dgrad + dgelu)
m, n, k = shapes["ff1"]
x, w, b = rnd(m, k), rnd(n, k), rnd(n)
aux = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
y = G.mm_nt(x, w, bias=b, gelu_aux=aux)
h = torch.addmm(b, x, w.t())
print("gelu epi: pre-act err", rel(aux, h.float()), "act err", rel(y, torch.nn.functional.gelu(h).float()))
dy2, w2t = rnd(m, d), rnd(n, d)
g = G.mm_nt(dy2, w2t, dgelu_aux=aux)
ref = torch.ops.aten.gelu_backward(dy2 @ w2t.t(), aux)
print("dgelu epi err", rel(g, ref.float()))
