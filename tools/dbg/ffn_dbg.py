"""ConvFFNFn / attention_qkv at the train.py-width C5 shapes (B=1, T=64,
d 512, FFN 1024, 2 heads of 64) against torch / the unfused paths.
python tools/dbg/ffn_dbg.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from mtts import convgemm as CG  # noqa: E402
from mtts import attn_kernels as AK  # noqa: E402

dev = "cuda"


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


for (B, T, C, H) in [(1, 64, 512, 1024), (3, 37, 512, 1024), (1, 64, 64, 128), (2, 64, 512, 1024), (1, 32, 512, 1024)]:
    torch.manual_seed(0)
    x = torch.randn(B, T, C, device=dev)
    w1, b1 = torch.randn(H, C, 9, device=dev) / 68, torch.randn(H, device=dev) * 0.1
    w2, b2 = torch.randn(C, H, 1, device=dev) / 32, torch.randn(C, device=dev) * 0.1
    g = torch.randn(B, T, C, device=dev)
    res = []
    for mode in ("fused", "torch"):
        ts = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
        if mode == "fused":
            y = CG.conv_ffn(*ts)
        else:
            h = torch.relu(F.conv1d(ts[0].transpose(1, 2), ts[1], ts[2], padding=4))
            y = F.conv1d(h, ts[3], ts[4]).transpose(1, 2)
        (y * g).sum().backward()
        res.append([y.detach()] + [t.grad for t in ts])
    print(f"FFN B{B} T{T} C{C} H{H}: " + ", ".join(f"{n} {rel(a, r):.1e}" for n, a, r in
                                                     zip(("y", "dx", "dw1", "db1", "dw2", "db2"), *res)), flush=True)
    d, nh = 128, 2
    qkv = torch.randn(B, T, 3 * d, device=dev)
    go = torch.randn(B, T, d, device=dev)
    outs = []
    for mode in ("qkv", "sep"):
        t = qkv.clone().requires_grad_(True)
        if mode == "qkv":
            o = AK.attention_qkv(t, nh)
        else:
            o = AK.attention(t[..., :d], t[..., d:2 * d], t[..., 2 * d:], nh)
        (o * go).sum().backward()
        outs.append([o.detach(), t.grad])
    print(f"  attention_qkv vs separate: out {rel(outs[0][0], outs[1][0]):.1e}, dqkv {rel(outs[0][1], outs[1][1]):.1e}",
          flush=True)
