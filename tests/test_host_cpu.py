"""Host-side pieces of the training step on CPU: clip-in-optimizer
(mtts/optim.py) against clip_grad_norm_ + the same optimizer.  (The
embedding sums run on the HIP kernel: tests/test_gpu_codec.py.)"""
import pytest
import torch
import torch.nn.functional as F


def test_clip_into_optimizer_equals_clip_grad_norm():
    from mtts.optim import clip_into_optimizer
    torch.manual_seed(0)
    try:
        torch.optim.Adam([torch.zeros(1, requires_grad=True)], fused=True)
    except Exception as e:  # pragma: no cover
        pytest.skip(f"fused Adam unavailable on CPU: {e}")
    ps1 = [torch.randn(7, 5, requires_grad=True), torch.randn(11, requires_grad=True)]
    ps2 = [p.detach().clone().requires_grad_(True) for p in ps1]
    o1 = torch.optim.Adam(ps1, lr=1e-2, fused=True)
    o2 = torch.optim.Adam(ps2, lr=1e-2, fused=True)
    for step in range(3):
        gs = [torch.randn_like(p) * 10 for p in ps1]
        for p, gg in zip(ps1, gs):
            p.grad = gg.clone()
        for p, gg in zip(ps2, gs):
            p.grad = gg.clone()
        n1 = torch.nn.utils.clip_grad_norm_(ps1, 1.0)
        o1.step()
        n2 = clip_into_optimizer(o2, ps2, 1.0)
        o2.step()
        torch.testing.assert_close(n1, n2)
        for a, b in zip(ps1, ps2):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
