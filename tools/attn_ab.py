"""Attention fwd/bwd timing at the C2 (T_kv=128) and C5 (T_kv=5248) shapes,
with the generic kernels and query-chunk counts forced through the library's
path overrides (mtts_set_override).  python tools/attn_ab.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_ROOT: another package tree (tools/ab/base) for a same-box A/B
sys.path[:0] = [ROOT, os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd")]
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


SHAPES = {"C2": (8, 2048, 128, 128), "C5": (4, 5120, 5248, 128), "C5m": (8, 5120, 5248, 64),
          # query-count probes of the workgroup-round tail at C5m (2048 / 2560 / 3072 workgroups)
          "C5m4k": (8, 4096, 5248, 64), "C5m6k": (8, 6144, 5248, 64)}
for name in os.environ.get("SHAPES", "C2,C5,C5m").split(","):
    B, T, S, hd = SHAPES[name]
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
    fl = 4 * B * T * S * d
    tf = timed(lambda: A.attention_fwd(q, k, v, H, kpm, want_lse=True))
    print(f"{name} fwd {tf * 1e3:.1f} us {fl / tf / 1e9:.0f} TF/s", flush=True)
    with L.override(attn_generic=1):
        tf0 = timed(lambda: A.attention_fwd(q, k, v, H, kpm, want_lse=True))
        o0, l0 = A.attention_fwd(q, k, v, H, kpm, want_lse=True)
    print(f"{name} fwd generic kernel {tf0 * 1e3:.1f} us {fl / tf0 / 1e9:.0f} TF/s; max|diff| out "
          f"{(o0.float() - out.float()).abs().max().item():.2e} lse {(l0 - lse).abs().max().item():.2e}", flush=True)
    for ch in ([None, 8, 16, 32] if name == "C2" else [None]):
        with L.override(attn_chunks=ch):
            tb = timed(lambda: A.attention_bwd(q, k, v, H, kpm, out, lse, do))
        print(f"{name} bwd chunks={ch} {tb * 1e3:.1f} us {2.5 * fl / tb / 1e9:.0f} TF/s", flush=True)
