"""A/B timing of selective_scan_fwd variants at the north-star shape.

python tools/scan_ab.py [variant ...]     (env MTTS_LIB selects a library build)

Inputs are allocated once per dtype; the variants (env switches read at each
launch) are interleaved over several rounds so clock drift hits all of them
alike; prints the median and best per-launch time of each."""
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import ops  # noqa: E402

VARIANTS = [("xl", {}), ("dpp", {"MTTS_SCAN_XDPP": "1"}), ("v1", {"MTTS_SCAN_FWD_V1": "1"}),
            ("p2", {"MTTS_SCAN_P": "2"}), ("p2k2", {"MTTS_SCAN_P": "2", "MTTS_SCAN_SEGS": "2"}),
            ("k2", {"MTTS_SCAN_SEGS": "2"}), ("p4", {"MTTS_SCAN_P": "4"}), ("w2", {"MTTS_SCAN_NO_C1": "1"}),
            ("c1small", {"MTTS_C1_SMALL": "1"})]
KEYS = ("MTTS_SCAN_FWD_V1", "MTTS_SCAN_XDPP", "MTTS_SCAN_P", "MTTS_SCAN_SEGS", "MTTS_SCAN_NO_C1", "MTTS_C1_SMALL")
sel = [a for a in sys.argv[1:] if not a.startswith("-")]
variants = [v for v in VARIANTS if not sel or v[0] in sel]
dtypes = (torch.bfloat16, torch.float32)
if "--bf16" in sys.argv:
    dtypes = (torch.bfloat16,)
if "--fp32" in sys.argv:
    dtypes = (torch.float32,)


def inputs(dtype, B=32, L=8192, D=2048, N=16):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    z = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    delta = (torch.randn(B, L, D, device=dev, generator=g) * 0.1).to(dtype)
    Bm = torch.randn(B, L, N, device=dev, generator=g).to(dtype)
    Cm = torch.randn(B, L, N, device=dev, generator=g).to(dtype)
    A = -torch.arange(1, N + 1, device=dev, dtype=torch.float32).repeat(D, 1)
    Dp = torch.ones(D, device=dev)
    dt0 = torch.exp(torch.rand(D, device=dev, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
    bias = dt0 + torch.log(-torch.expm1(-dt0))
    out = torch.empty_like(u)
    es = torch.finfo(dtype).bits // 8
    nbytes = 4 * B * D * L * es + 2 * B * N * L * es + (D * N + 2 * D) * 4
    return (u, delta, A, Bm, Cm, Dp, z, bias, True), out, nbytes


for dtype in dtypes:
    args, out, nbytes = inputs(dtype)
    times = {n: [] for n, _ in variants}
    for rnd in range(5):
        for name, env in variants:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(3):
                ops.scan_fwd(*args, out=out)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(20):
                ops.scan_fwd(*args, out=out)
            ev[1].record()
            ev[1].synchronize()
            times[name].append(ev[0].elapsed_time(ev[1]) / 20)
    for name, _ in variants:
        med, best = statistics.median(times[name]), min(times[name])
        print(f"{name:5s} {str(dtype)[6:]:9s} north-star median {med:.3f} ms best {best:.3f} ms "
              f"{nbytes / med / 1e6:.0f} GB/s ({nbytes / med / 8e9 * 100:.1f}% of 8 TB/s)", flush=True)
    del args, out
    torch.cuda.empty_cache()
