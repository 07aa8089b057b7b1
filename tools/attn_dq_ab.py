"""Same-process A/B of the long-key attention backward's dQ staging (override
attn_dq_dma: 0 register-staged K / V blocks, 1 LDS-DMA ring) at the C5 shapes,
interleaved rounds.  python tools/attn_dq_ab.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import _lib as L  # noqa: E402
from mtts import attn_kernels as A  # noqa: E402


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


for name, (B, T, S, hd) in (("C5m", (8, 5120, 5248, 64)),):
    H = 8
    d = H * hd
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, T, d, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(B, S, d, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(B, S, d, device="cuda", generator=g).to(torch.bfloat16)
    kpm = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    kpm[:, int(S * 0.9):] = True
    out, lse = A.attention_fwd(q, k, v, H, kpm, want_lse=True)
    do = torch.randn_like(out)
    for rnd in range(3):
        for dma in (0, 1):
            with L.override(attn_bwd=L.ATTN_BWD_SPLIT, attn_dq_dma=dma):
                tb = timed(lambda: A.attention_bwd(q, k, v, H, kpm, out, lse, do))
            print(f"{name} round {rnd} dq_dma={dma} bwd (dQ + dK/dV) {tb * 1e3:.1f} us", flush=True)
