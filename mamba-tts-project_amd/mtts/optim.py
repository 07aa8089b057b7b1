"""Gradient-norm clipping folded into a fused optimizer step.

torch.nn.utils.clip_grad_norm_(params, max_norm) (the reference training
step, train.py) computes the global L2 norm and then rewrites every gradient
(`g *= min(1, max_norm / (norm + 1e-6))`), a full read+write pass over all
gradients.  torch's fused Adam/AdamW divide every gradient by an optional
device scalar `grad_scale` inside their single pass, so the same update is
obtained by computing the norm (one read pass) and handing the optimizer
`grad_scale = 1 / clip_coef` -- one HBM pass over the gradients instead of
two.  Gradients themselves are left unclipped.
"""
from __future__ import annotations

import torch


@torch.no_grad()
def clip_into_optimizer(optimizer, params, max_norm: float, eps: float = 1e-6):
    """Return the total gradient norm; arm `optimizer` (fused Adam/AdamW) to
    apply clip_grad_norm_'s scaling in its next step()."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.zeros(())
    norms = torch._foreach_norm(grads, 2.0)
    total = torch.linalg.vector_norm(torch.stack([n.float() for n in norms]), 2.0)
    coef = torch.clamp(max_norm / (total + eps), max=1.0)
    scale = getattr(optimizer, "grad_scale", None)
    if scale is None or scale.device != total.device:
        optimizer.grad_scale = torch.empty((), device=total.device, dtype=torch.float32)
    optimizer.grad_scale.copy_(1.0 / coef)
    return total
