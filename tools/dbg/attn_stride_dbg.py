"""fp32 attention with q / k / v as strided thirds of one (B, T, 3d) tensor vs
contiguous copies vs an fp64 softmax reference (the text encoder's fused
q/k/v path).   python tools/dbg/attn_stride_dbg.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import attn_kernels as AK  # noqa: E402


def ref(q, k, v, H, kpm):
    B, T, d = q.shape
    hd = d // H
    qh, kh, vh = (t.double().view(B, -1, H, hd).transpose(1, 2) for t in (q, k, v))
    s = qh @ kh.transpose(-1, -2) / hd ** 0.5
    if kpm is not None:
        s = s.masked_fill(kpm[:, None, None, :], float("-inf"))
    return (s.softmax(-1) @ vh).transpose(1, 2).reshape(B, T, d)


for B, T, d, H, pad in [(1, 64, 128, 2, 0), (3, 37, 128, 2, 9), (1, 64, 32, 2, 0), (2, 100, 128, 2, 0), (1, 200, 128, 2, 0)]:
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * d, device="cuda")
    kpm = torch.zeros(B, T, dtype=torch.bool, device="cuda")
    if pad:
        kpm[1:, T - pad:] = True
    q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    o_s = AK.attention_fwd(q, k, v, H, kpm)[0]
    o_c = AK.attention_fwd(q.contiguous(), k.contiguous(), v.contiguous(), H, kpm)[0]
    r = ref(q, k, v, H, kpm)
    e = lambda a: ((a.double() - r).abs().max() / r.abs().max()).item()  # noqa: E731
    print(f"B{B} T{T} d{d} H{H} pad{pad}: strided {e(o_s):.1e}  contiguous {e(o_c):.1e}", flush=True)
