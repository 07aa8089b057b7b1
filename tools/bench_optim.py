"""Optimizer step at the C2 parameter count: FusedClipAdam (mtts_clip_adam)
vs torch fused Adam + foreach-norm clip (clip_into_optimizer)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import mamba_decoder  # noqa: E402
from mtts.optim import FusedClipAdam, clip_into_optimizer  # noqa: E402

m = mamba_decoder.MambaTTSDecoder(10, d_model=1024, n_layers=12, n_heads=8, d_ff=2048, d_style=256).cuda()
ps = list(m.parameters())
n = sum(p.numel() for p in ps)
for p in ps:
    p.grad = torch.randn_like(p) * 1e-3


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(it):
        fn()
    e[1].record()
    e[1].synchronize()
    return e[0].elapsed_time(e[1]) / it


a = FusedClipAdam(ps, lr=1e-4, max_grad_norm=1.0)
t1 = timed(a.step)
b = torch.optim.Adam(ps, lr=1e-4, fused=True)
t2 = timed(lambda: (clip_into_optimizer(b, ps, 1.0), b.step()))
print(f"params {n / 1e6:.1f} M: FusedClipAdam {t1:.3f} ms ({32 * n / t1 / 1e9:.2f} TB/s at 32 B/param), "
      f"torch fused Adam + foreach clip {t2:.3f} ms; uploads {[q['uploads'] for q in a._plans.values()]}")
