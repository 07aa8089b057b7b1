"""wgrad formulations for C2 shapes: dW[n,k] = dy[M,n]^T @ x[M,k]."""
import torch
M = 16384
shapes = {"in_proj": (4096, 1024), "x_proj": (96, 2048), "dt_proj": (2048, 64), "out_proj": (1024, 2048),
          "q_proj": (1024, 1024), "ff1": (2048, 1024), "ff2": (1024, 2048)}
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3
has_od = True
try:
    a = torch.randn(64, 64, device="cuda", dtype=torch.bfloat16)
    torch.mm(a, a, out_dtype=torch.float32)
except Exception as e:
    has_od = False; print("no out_dtype:", e)
for name, (n, k) in shapes.items():
    dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * n * k
    res = {"base": t(lambda: dy.t() @ x)}
    for s in (4, 8, 16):
        res[f"bmm{s}"] = t(lambda: torch.bmm(dy.view(s, M // s, n).transpose(1, 2), x.view(s, M // s, k)).sum(0))
        if has_od:
            res[f"bmm{s}f"] = t(lambda: torch.bmm(dy.view(s, M // s, n).transpose(1, 2), x.view(s, M // s, k), out_dtype=torch.float32).sum(0))
    if has_od:
        res["mm_f32"] = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    dyt = dy.t().contiguous()
    res["contigT"] = t(lambda: dyt @ x)
    best = min(res, key=res.get)
    print(f"{name:9s} " + " ".join(f"{kk}={v:6.1f}" for kk, v in res.items()) + f"  best={best} {fl/res[best]/1e6:.0f}TF", flush=True)
