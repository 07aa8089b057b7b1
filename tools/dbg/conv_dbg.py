import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import numpy as np, torch
from mtts import _lib, ops
g = np.load(os.path.join(ROOT, "tests/golden/conv1d.npz"))
for (B, L, D, dt) in [(2, 64, 64, torch.float32), (2, 64, 256, torch.float32), (2, 64, 2048, torch.float32),
                      (2, 64, 64, torch.bfloat16), (1, 40, 1024, torch.float32)]:
    torch.manual_seed(0)
    x = torch.randn(B, L, D, device="cuda").to(dt)
    w = torch.randn(D, 4, device="cuda"); b = torch.randn(D, device="cuda")
    with _lib.override(conv_untiled=1):
        r, _ = ops.conv_fwd(x, w, b, True)
    o, _ = ops.conv_fwd(x, w, b, True)
    bad = (o.float() - r.float()).abs() > 1e-3 * r.float().abs().max()
    idx = bad.nonzero()
    print(B, L, D, dt, "bad", int(bad.sum()), "of", bad.numel())
    if len(idx):
        ts = sorted(set(idx[:, 1].tolist())); cs = sorted(set(idx[:, 2].tolist()))
        print("  rows", ts[:40], "\n  cols", cs[:40] if len(cs) < 80 else (cs[:20], "...", len(cs)))
        # which reference row does the wrong value equal?
        bb, t, c = idx[0].tolist()
        col = r[bb, :, c].float()
        hit = ((col - o[bb, t, c].float()).abs() < 1e-5).nonzero().flatten().tolist()
        print("  first bad", (bb, t, c), "equals ref rows", hit)
