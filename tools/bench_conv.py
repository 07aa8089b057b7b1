"""Causal conv1d fwd / bwd at the C2 shape (B=8, L=2048, d_inner=2048 bf16,
x a strided view of xz as in the decoder): time and HBM rate."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_ROOT: another package tree (tools/ab/base) for a same-box A/B
sys.path[:0] = [ROOT, os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import _lib, ops  # noqa: E402

B, L, D = 8, 2048, 2048
xz = torch.randn(B, L, 2 * D, device="cuda").to(torch.bfloat16)
x = xz[..., :D]
w = torch.randn(D, 1, 4, device="cuda") * 0.3
bias = torch.randn(D, device="cuda") * 0.1
du = torch.randn(B, L, D, device="cuda").to(torch.bfloat16)
dxz = torch.empty_like(xz)


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
    return e0.elapsed_time(e1) / it * 1e3


n = B * L * D * 2
for rnd in range(2):
    for mode in ("tiled", "untiled"):
        with _lib.override(conv_untiled=int(mode == "untiled")):
            tf = t(lambda: ops.conv_fwd(x, w, bias, True))
            tb = t(lambda: ops.conv_bwd(x, w, bias, du, True, dx=dxz[..., :D]))
        print(f"{mode:8s} conv fwd {tf:.1f} us ({2 * n / tf / 1e3:.0f} GB/s)   bwd {tb:.1f} us "
              f"({3 * n / tb / 1e3:.0f} GB/s)", flush=True)
