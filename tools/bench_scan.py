"""Sweep the selective-scan kernels: P (lanes per channel), dtype, shapes."""
import math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch
from mtts import ops

def inputs(B, L, D, dtype, dev="cuda"):
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    z = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    dl = (torch.randn(B, L, D, device=dev, generator=g) * 0.1).to(dtype)
    Bm = torch.randn(B, L, 16, device=dev, generator=g).to(dtype)
    Cm = torch.randn(B, L, 16, device=dev, generator=g).to(dtype)
    A = -torch.arange(1, 17, device=dev, dtype=torch.float32).repeat(D, 1)
    Dp = torch.ones(D, device=dev)
    bias = torch.full((D,), -3.0, device=dev)
    return u, dl, A, Bm, Cm, Dp, z, bias

def timeit(fn, iters=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / iters

shapes = [(32, 8192, 2048), (8, 2048, 2048)]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    shapes = [(8, 2048, 2048)]
for (B, L, D) in shapes:
    for dtype in (torch.bfloat16, torch.float32):
        u, dl, A, Bm, Cm, Dp, z, bias = inputs(B, L, D, dtype)
        es = torch.finfo(dtype).bits // 8
        nbytes = 4 * B * D * L * es + 2 * B * 16 * L * es
        out = torch.empty_like(u)
        for P in ("2", "4"):
            os.environ["MTTS_SCAN_P"] = P
            ms = timeit(lambda: ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, out=out))
            print(f"fwd B={B} L={L} D={D} {str(dtype)[6:]} P={P}: {ms:.3f} ms  {nbytes/ms/1e6:.0f} GB/s  "
                  f"{B*L*D/ms/1e6:.1f} Gelem/s", flush=True)
        del os.environ["MTTS_SCAN_P"]
        if B * L * D <= 8 * 2048 * 2048:
            _, _, ck = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_ckpt=True)
            go = torch.randn_like(u)
            ms = timeit(lambda: ops.scan_bwd(u, dl, A, Bm, Cm, Dp, z, bias, True, None, ck, go), 5)
            print(f"bwd B={B} L={L} D={D} {str(dtype)[6:]}: {ms:.3f} ms", flush=True)
        del u, dl, z, Bm, Cm, out
        torch.cuda.empty_cache()
