"""Per-shape timing of the fp32 windowed-row GEMM (mtts_convgemm) on the
text-encoder bench leg's convolutions / projections (B=8, 128 phonemes,
d 512, FFN 1024 k=9, duration filter 256 k=3) against torch (hipBLASLt /
MIOpen) on the same shapes.   python tools/convgemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from mtts import convgemm as CG  # noqa: E402


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
    return e0.elapsed_time(e1) / it * 1e3


B, T = 8, 128
if os.environ.get("SPLITS"):   # fixed split count for every GEMM (heuristic check)
    CG.FORCE_SPLITS = int(os.environ["SPLITS"])
    print("splits", CG.FORCE_SPLITS, flush=True)
if os.environ.get("HALO") == "0":   # explicit zero-padded copies instead of halo row maps (A/B)
    CG._halo_ok = lambda C_, p: False
    print("halo off", flush=True)
for (C, O, K) in [(512, 1024, 9), (1024, 512, 1), (512, 384, 1), (128, 512, 1), (512, 256, 3), (256, 256, 3)]:
    x = torch.randn(B, T, C, device="cuda")
    w = torch.randn(O, C, K, device="cuda") / (C * K) ** 0.5
    b = torch.randn(O, device="cuda")
    dy = torch.randn(B, T, O, device="cuda")
    y, xp, wf = CG.conv_forward(x, w, b, False)
    fl = 2.0 * B * T * O * C * K
    t_f = timed(lambda: CG.conv_forward(x, w, b, False))
    t_dx = timed(lambda: CG.conv_backward(dy, xp, wf, K, True, False, False))
    t_dw = timed(lambda: CG.conv_backward(dy, xp, wf, K, False, True, False))
    xt = x.transpose(1, 2).contiguous()
    t_tf = timed(lambda: F.conv1d(xt, w, b, padding=(K - 1) // 2))
    print(f"C{C} O{O} K{K}: fwd {t_f:6.1f} us {fl / t_f / 1e6:5.1f} TF/s | dgrad {t_dx:6.1f} us {fl / t_dx / 1e6:5.1f} | "
          f"wgrad {t_dw:6.1f} us {fl / t_dw / 1e6:5.1f} | torch conv fwd {t_tf:6.1f} us {fl / t_tf / 1e6:5.1f}", flush=True)
