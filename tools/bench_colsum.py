"""Bias-gradient column sums (mtts_colsum, 16384 token rows) at the C2 widths:
per-call time for row-chunk sizes (MTTS_COLSUM_RCHUNK), interleaved."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts.linear import colsum  # noqa: E402


def t(fn, it=50):
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


for cols in (1024, 2048, 3072):
    x = torch.randn(16384, cols, device="cuda").to(torch.bfloat16)
    ref = x.float().sum(0)
    line = f"cols {cols}:"
    for rc in ("128", "64", "32", "64", "128"):
        os.environ["MTTS_COLSUM_RCHUNK"] = rc
        out = colsum(x)
        assert ((out - ref).abs().max() / ref.abs().max()).item() < 1e-5
        line += f"  rchunk {rc} {t(lambda: colsum(x)):6.1f} us"
    print(line, flush=True)
