"""Run the C2-shape selective-scan backward (B=8, L=2048, d_inner=2048, bf16
I/O) ITERS times after one forward, for rocprofv3 kernel traces / PMC passes.
python tools/scan_bwd_once.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import ops  # noqa: E402

B, L, D = 8, 2048, 2048
g = torch.Generator(device="cuda").manual_seed(0)
u, z = (torch.randn(B, L, D, device="cuda", generator=g).bfloat16() for _ in range(2))
dl = (torch.randn(B, L, D, device="cuda", generator=g) * 0.1).bfloat16()
Bm, Cm = (torch.randn(B, L, 16, device="cuda", generator=g).bfloat16() for _ in range(2))
A = -torch.arange(1, 17, device="cuda", dtype=torch.float32).repeat(D, 1)
a = (u, dl, A, Bm, Cm, torch.ones(D, device="cuda"), z, torch.full((D,), -4.0, device="cuda"))
_, _, ck = ops.scan_fwd(*a, True, want_ckpt=True)
dout = torch.randn_like(a[0])
for _ in range(int(os.environ.get("ITERS", "5"))):
    ops.scan_bwd(*a, True, None, ck, dout)
torch.cuda.synchronize()
print("scan bwd done", flush=True)
