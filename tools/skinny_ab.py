"""Skinny GEMMs (csrc/skinny.hip) vs torch/hipBLASLt at the C2 Mamba shapes
(per-op event timings), then the in-process C2 training step with the skinny
routing on / off (gemm.SKINNY, gemm.SKINNY_TN_KERNEL), interleaved rounds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_ROOT: another package tree (tools/ab/base) for a same-box A/B
sys.path[:0] = [ROOT, os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402
from mtts import linear as LIN  # noqa: E402


def t(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def op_bench():
    M, D, R = 16384, 2048, 64
    bf = torch.bfloat16
    u = torch.randn(M, D, device="cuda").to(bf)
    wx = torch.randn(R + 32, D, device="cuda").to(bf)
    wdt = torch.randn(D, R, device="cuda").to(bf)
    x_dbl = torch.randn(M, R + 32, device="cuda").to(bf)
    dd = torch.randn(M, D, device="cuda").to(bf)
    dx = torch.zeros(M, R + 32, device="cuda")
    du = torch.randn(M, D, device="cuda").to(bf)
    wdt_t, wx_t = wdt.t().contiguous(), wx.t().contiguous()
    gx = x_dbl
    ops = {
        "x_proj fwd  (16384x96, K=2048)": (lambda: G.mm_skinny(u, wx), lambda: u @ wx.t()),
        "dt_proj fwd (16384x2048, K=64)": (lambda: G.mm_skinny(x_dbl[:, :R], wdt), lambda: x_dbl[:, :R] @ wdt.t()),
        "d(dt)       (16384x64, K=2048)": (lambda: G.mm_skinny(dd, wdt_t, out=dx[:, :R]),
                                           lambda: dx[:, :R].copy_(dd @ wdt)),
        "du += gx Wx (16384x2048, K=96)": (lambda: G.mm_skinny(gx, wx_t, out=du, beta=1.0), lambda: du.addmm_(gx, wx)),
    }
    for name, (a, b) in ops.items():
        print(f"{name}: skinny {t(a):6.1f} us   torch {t(b):6.1f} us", flush=True)
    for name, (dy_, x_) in {"dW_dt (2048x64)": (dd, x_dbl[:, :R]), "dW_x (96x2048)": (gx, u)}.items():
        G.WGRAD_SKINNY_ON_TN = True
        a = t(lambda: LIN.wgrad(dy_, x_))
        G.WGRAD_SKINNY_ON_TN = False
        b = t(lambda: LIN.wgrad(dy_, x_))
        print(f"{name}: TN {a:6.1f} us   bmm split {b:6.1f} us", flush=True)
    for name, (a_, b_, tr) in {"dW_dt skinny-TN": (dd, x_dbl[:, :R], False), "dW_x^T skinny-TN": (u, gx, True)}.items():
        print(f"{name}: {t(lambda: G.mm_skinny_tn(a_, b_, trans_c=tr)):6.1f} us", flush=True)


import bench  # noqa: E402
import mamba_decoder  # noqa: E402
from mtts.optim import FusedClipAdam  # noqa: E402

c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)
opt = FusedClipAdam(list(model.parameters()), lr=1e-4, max_grad_norm=1.0)


def step():
    logits = model(tokens, text, z, text_mask=mask)
    loss = torch.nn.functional.cross_entropy(logits.float().view(-1, c["vocab"]), tokens.view(-1), ignore_index=0)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()


def timeit(n=10):
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


if __name__ == "__main__":
    op_bench()
    if len(sys.argv) > 1 and sys.argv[1] == "ops":
        sys.exit(0)
    res = {"skinny": [], "skinny+xproj": [], "skinny-du": [], "skinny-du-dtproj": [], "off": []}
    for _ in range(3):
        for kind in res:
            G.SKINNY = kind != "off"
            G.SKINNY_XPROJ = kind == "skinny+xproj"
            G.SKINNY_DU = kind not in ("skinny-du", "skinny-du-dtproj")
            G.SKINNY_DTPROJ = kind != "skinny-du-dtproj"
            res[kind].append(timeit())
    print({k: [round(x, 2) for x in v] for k, v in res.items()}, flush=True)
