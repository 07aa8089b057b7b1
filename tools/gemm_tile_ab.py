"""Same-process A/B of the NT GEMM tiles (gemm_tile override: 1 = eight-wave
ping-pong, 2 = four-wave 128x128 per wave) on every C2 forward / data-gradient
shape, interleaved rounds, HIP-event timing; with a max-error check of each
tile against an fp32 product.   python tools/gemm_tile_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import _lib as L  # noqa: E402
from mtts import gemm as G  # noqa: E402

M = 8 * 2048
SHAPES = {  # name: (m, n, k, epilogue)
    "in_proj fwd": (M, 4096, 1024, None), "out_proj fwd": (M, 1024, 2048, None), "q/o fwd": (M, 1024, 1024, "bias"),
    "ff1 fwd": (M, 2048, 1024, "gelu"), "ff2 fwd": (M, 1024, 2048, "bias"),
    "in_proj dgrad": (M, 1024, 4096, None), "out_proj dgrad": (M, 2048, 1024, None), "ff2 dgrad": (M, 2048, 1024, "dgelu"),
    "ff1 dgrad": (M, 1024, 2048, None), "big 8192": (M, 4096, 8192, None),
}
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 3


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


tot = {1: 0.0, 2: 0.0}
for name, (m, n, k, epi) in SHAPES.items():
    torch.manual_seed(0)
    a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
    bias = torch.randn(n, device="cuda") if epi in ("bias", "gelu") else None
    aux = torch.empty(m, n, device="cuda", dtype=torch.bfloat16) if epi == "gelu" else None
    daux = torch.randn(m, n, device="cuda").bfloat16() if epi == "dgelu" else None
    out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)

    def run():
        G.mm_nt(a, b, bias=bias, gelu_aux=aux, dgelu_aux=daux, out=out)

    ref = a.float() @ b.float().t()
    errs = {}
    for tile in (1, 2):
        with L.override(gemm_tile=tile):
            G.mm_nt(a, b, out=out)
            errs[tile] = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    best = {1: 1e9, 2: 1e9}
    for _ in range(ROUNDS):
        for tile in (1, 2):
            with L.override(gemm_tile=tile):
                best[tile] = min(best[tile], timed(run))
    fl = 2.0 * m * n * k
    for t in (1, 2):
        if name != "big 8192":
            tot[t] += best[t]
    print(f"{name:15s} {m}x{n}x{k} {epi or '':5s} pingpong {best[1] * 1e3:7.1f} us {fl / best[1] / 1e9:6.0f} TF/s | "
          f"fourwave {best[2] * 1e3:7.1f} us {fl / best[2] / 1e9:6.0f} TF/s | ratio {best[1] / best[2]:.3f} | "
          f"err {errs[1]:.1e} / {errs[2]:.1e}", flush=True)
print(f"sum over the C2 shapes: pingpong {tot[1] * 1e3:.1f} us, fourwave {tot[2] * 1e3:.1f} us", flush=True)
