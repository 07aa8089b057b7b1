"""LayerNorm fwd / bwd timing at the C2 shape (16384 x 1024 bf16, FiLM per
2048-row group, fused residual, dx accumulate).
python tools/bench_ln.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_ROOT: another package tree (tools/ab/base) for a same-box A/B
sys.path[:0] = [ROOT, os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import ops  # noqa: E402


def timed(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(it):
        fn()
    e[1].record()
    e[1].synchronize()
    return e[0].elapsed_time(e[1]) / it * 1e3


rows, cols, T = 16384, 1024, 2048
bf = torch.bfloat16
x = torch.randn(rows, cols, device="cuda").to(bf)
res = torch.randn(rows, cols, device="cuda").to(bf)
w = torch.randn(cols, device="cuda")
b = torch.randn(cols, device="cuda")
gamma = torch.randn(rows // T, cols, device="cuda")
beta = torch.randn(rows // T, cols, device="cuda")
dy = torch.randn(rows, cols, device="cuda").to(bf)
acc = torch.randn(rows, cols, device="cuda").to(bf)
y, mean, rstd, xs = ops.layernorm_fwd(x, w, b, 1e-5, res=res, gamma=gamma, beta=beta, rows_per_group=T)
tf = timed(lambda: ops.layernorm_fwd(x, w, b, 1e-5, res=res, gamma=gamma, beta=beta, rows_per_group=T))
print(f"fwd (x+res, FiLM, x_sum): {tf:.1f} us  {4 * rows * cols * 2 / tf / 1e3:.0f} GB/s", flush=True)
tb = timed(lambda: ops.layernorm_bwd(xs, w, b, 1e-5, gamma, beta, T, mean, rstd, dy, dx_acc=acc))
print(f"bwd (FiLM, dx_acc): {tb:.1f} us  {4 * rows * cols * 2 / tb / 1e3:.0f} GB/s (x, dy, acc, dx)", flush=True)
