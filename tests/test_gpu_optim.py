"""GPU parity of the fused clip + Adam step (mtts_clip_adam, SURVEY.md §8f
row 4) against the reference's own optimizer path: torch.nn.utils.
clip_grad_norm_ + torch.optim.Adam (train.py:152-158, 232-235), run on the
CPU in float64 with the same parameters and gradients, over several steps.
Tolerance: norm, exp_avg, exp_avg_sq 1e-5 relative; parameters 1e-4 of
max|p| -- an fp32 update lr*m/(sqrt(v)+eps) differs from the float64 one by
up to ~1e-2*lr where weight decay cancels a gradient down to ~eps (the
fp32 rounding of g is then a large part of it)."""
import pytest
import torch

from test_gpu_ops import close, DEV

pytestmark = pytest.mark.gpu

SHAPES = [(4096, 1024), (7,), (65537,), (96, 2048), (3, 5, 2), (1,)]


@pytest.mark.parametrize("max_norm", [1.0, None, 1e6])
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_clip_adam_vs_torch(max_norm, wd):
    from mtts.optim import FusedClipAdam
    torch.manual_seed(0)
    init = [torch.randn(*s) for s in SHAPES]
    gp = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    cp = [torch.nn.Parameter(t.clone().double()) for t in init]
    opt = FusedClipAdam(gp, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=wd, max_grad_norm=max_norm)
    ref = torch.optim.Adam(cp, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=wd)
    for step in range(4):
        grads = [torch.randn(*s) * (3.0 if step % 2 else 0.01) for s in SHAPES]
        for p, g in zip(gp, grads):
            p.grad = g.clone().to(DEV)
        for p, g in zip(cp, grads):
            p.grad = g.clone().double()
        total = None
        if max_norm is not None:
            total = torch.nn.utils.clip_grad_norm_(cp, max_norm)
        opt.step()
        ref.step()
        if total is not None:
            close(opt.last_grad_norm, total, rtol=1e-5, name="norm")
        for i, (a, b) in enumerate(zip(gp, cp)):
            close(a, b.detach(), rtol=1e-4, name=f"param{i} step{step}")
            close(opt.state[a]["exp_avg"], ref.state[b]["exp_avg"], rtol=1e-5, name=f"m{i}")
            close(opt.state[a]["exp_avg_sq"], ref.state[b]["exp_avg_sq"], rtol=1e-5, name=f"v{i}")
    assert float(opt.state[gp[0]]["step"]) == 4.0
    # state_dict interchange with torch.optim.Adam
    sd = opt.state_dict()
    t = torch.optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in gp], lr=1e-2)
    t.load_state_dict(sd)


def test_fused_clip_adam_rejects_mixed_steps():
    from mtts.optim import FusedClipAdam
    a = torch.nn.Parameter(torch.randn(8, device=DEV))
    b = torch.nn.Parameter(torch.randn(8, device=DEV))
    opt = FusedClipAdam([a, b], lr=1e-3)
    a.grad = torch.randn(8, device=DEV)
    opt.step()                       # only a steps
    a.grad = torch.randn(8, device=DEV)
    b.grad = torch.randn(8, device=DEV)
    with pytest.raises(ValueError, match="step count"):
        opt.step()


def test_fused_clip_adam_permuted_dense_parameter():
    """A conv weight kept [O][K][C] behind its (O, C, K) shape (text_encoder.
    kc_major): the step walks storage order, so p, grad and moments must share
    the layout -- result equal to the contiguous parameter's step; a gradient
    of another layout is refused."""
    from mtts.optim import FusedClipAdam
    torch.manual_seed(1)
    w0 = torch.randn(64, 32, 9, device=DEV)
    g0 = torch.randn(64, 32, 9, device=DEV)
    a = torch.nn.Parameter(w0.permute(0, 2, 1).contiguous().permute(0, 2, 1))
    b = torch.nn.Parameter(w0.clone())
    assert not a.is_contiguous()
    for p in (a, b):
        p.grad = torch.empty_like(p).copy_(g0)          # empty_like keeps the parameter's strides
    oa, ob = FusedClipAdam([a], lr=1e-2, max_grad_norm=1.0), FusedClipAdam([b], lr=1e-2, max_grad_norm=1.0)
    for _ in range(2):
        oa.step()
        ob.step()
    assert torch.equal(a.detach(), b.detach())
    assert opt_state_strides_match(oa, a)
    a.grad = g0.clone()                                  # contiguous gradient on the permuted parameter
    with pytest.raises(ValueError, match="same strides"):
        oa.step()


def opt_state_strides_match(opt, p):
    st = opt.state[p]
    return st["exp_avg"].stride() == p.stride() and st["exp_avg_sq"].stride() == p.stride()
