"""The k = 9 text-encoder convolution (B=8 x 128 tokens, 512 -> 1024) forward,
data gradient and weight gradient, ITERS times each, for rocprofv3 PMC passes
over the fp32 conv GEMM.   ITERS=5 python tools/convgemm_once.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import convgemm as CG  # noqa: E402

B, T, C, O, K = 8, 128, 512, 1024, 9
x = torch.randn(B, T, C, device="cuda")
w = torch.randn(O, C, K, device="cuda") / (C * K) ** 0.5
b = torch.randn(O, device="cuda")
dy = torch.randn(B, T, O, device="cuda")
y, xp, wf = CG.conv_forward(x, w, b, False)
for _ in range(int(os.environ.get("ITERS", "5"))):
    CG.conv_forward(x, w, b, False)
    CG.conv_backward(dy, xp, wf, K, True, False, False)
    CG.conv_backward(dy, xp, wf, K, False, True, True)
torch.cuda.synchronize()
print("ok")
