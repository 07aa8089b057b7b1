"""Dropout on the HIP kernel (csrc/dropout.hip, mtts_dropout).

Replaces nn.Dropout / F.dropout in the training paths of the drop-in modules
(reference style_cross_attention.py:38-46, 100-109, 133, 246-255, 278 and the
FastSpeech2 blocks behind text_encoder.py:80-85, 168).  The mask is
counter-based (a hash of a per-call seed and the element index), so nothing
is stored for the backward: it regenerates the mask from the same seed.
Seeds come from torch's default CPU generator (torch.manual_seed reproduces
a run; no device sync), plus a per-device int64 base in HBM that `advance()`
moves (a captured add): a training step captured in a hipGraph -- whose CPU
seeds are frozen at capture -- draws fresh masks on every replay when it
calls `advance()` first.  The forward records the base it used in a per-call
device slot that its backward reads, so advancing between a forward and its
backward cannot desynchronise the two masks.  The masks are not torch's (no two implementations'
dropout draws match element for element); the keep probability and scale
are: keep with probability 1 - p, survivors scaled by 1 / (1 - p).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


def new_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


_base = {}


def device_base(device) -> torch.Tensor:
    """The per-device int64 seed base (HBM) every training-mode mask adds."""
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _base.get(key)
    if t is None:
        t = _base[key] = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", key))
    return t


def advance(device=None) -> None:
    """Move the device seed base (one small kernel; capturable): call once
    per training step when the step is replayed from a hipGraph."""
    t = device_base(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    t.add_(0x2545F4914F6CDD1D)     # odd: successive bases never repeat (mod 2^64)


def _slot(x):
    return device_base(x.device), torch.empty(1, dtype=torch.int64, device=x.device)


def _ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
            and t.numel() % 8 == 0 and t.data_ptr() % 16 == 0)


def apply_mask(x: torch.Tensor, p: float, seed: int, pre: torch.Tensor = None, out: torch.Tensor = None,
               group: int = 1, rep: int = 1, seed_in: torch.Tensor = None, seed_out: torch.Tensor = None):
    """y = x * keep(seed [+ *seed_in]) / (1 - p) [* gelu'(pre)] on the HIP
    kernel; one mask draw per `group` consecutive elements.  `rep` > 1: x
    (O, C) is broadcast to y (O, rep, C) (y[o, r] drops x[o]) without a copy.
    `seed_in` / `seed_out`: device int64 base added to the seed / where the
    kernel records it (forward -> backward)."""
    if not _ok(x):
        raise ValueError(f"dropout: contiguous 16-byte-aligned fp32/bf16 CUDA tensor with numel % 8 == 0 expected "
                         f"(got {x.dtype}, {tuple(x.shape)}, contiguous={x.is_contiguous()})")
    if pre is not None and (pre.dtype != torch.bfloat16 or pre.numel() != x.numel() or not _ok(pre)):
        raise ValueError("dropout: pre must be a contiguous bf16 tensor of x's size")
    if rep > 1:
        inner = x.shape[-1]
        y = torch.empty(x.numel() // inner, rep, inner, device=x.device, dtype=x.dtype) if out is None else out
        if y.numel() != x.numel() * rep or not y.is_contiguous():
            raise ValueError("dropout: broadcast output must be a contiguous (O, rep, C) tensor")
    else:
        y = torch.empty_like(x) if out is None else out
    a = L.DropoutArgs()
    a.n, a.dtype, a.p, a.seed = y.numel(), L.dtype_code(x), float(p), seed & (2 ** 64 - 1)
    a.x, a.y = x.data_ptr(), y.data_ptr()
    a.pre = 0 if pre is None else pre.data_ptr()
    a.group = group
    a.x_rep, a.x_inner = (rep, x.shape[-1]) if rep > 1 else (1, 0)
    a.seed_in, a.seed_out = L.ptr(seed_in), L.ptr(seed_out)
    L.call("mtts_dropout", a)
    return y


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, group=1):
        ctx.p, ctx.seed, ctx.group = p, new_seed(), group
        base, ctx.used = _slot(x)
        return apply_mask(x.contiguous(), p, ctx.seed, group=group, seed_in=base, seed_out=ctx.used)

    @staticmethod
    def backward(ctx, dy):
        return apply_mask(dy.contiguous(), ctx.p, ctx.seed, group=ctx.group, seed_in=ctx.used), None, None


class BcastDropoutFn(torch.autograd.Function):
    """dropout(x[:, None, :].expand(O, rep, C)) in one HIP pass (x (O, C));
    backward: the same mask on dy, then the column sums over each o's rep rows
    (mtts_colsum, fp32) -- the expand's gradient."""

    @staticmethod
    def forward(ctx, x, rep, p, group):
        ctx.p, ctx.seed, ctx.group, ctx.rep = p, new_seed(), group, rep
        ctx.xmeta = (x.shape, x.dtype)
        base, ctx.used = _slot(x)
        return apply_mask(x.contiguous(), p, ctx.seed, group=group, rep=rep, seed_in=base, seed_out=ctx.used)

    @staticmethod
    def backward(ctx, dy):
        from .linear import colsum_groups
        O, R, Cn = dy.shape
        g = apply_mask(dy.contiguous(), ctx.p, ctx.seed, group=ctx.group, seed_in=ctx.used)
        dx = colsum_groups(g.view(O * R, Cn), R).to(ctx.xmeta[1]).view(ctx.xmeta[0])
        return dx, None, None, None


def dropout_bcast(x: torch.Tensor, rep: int, p: float, group: int = 1) -> torch.Tensor:
    """Training-mode dropout of x (O, C) broadcast to (O, rep, C) (e.g. one
    value row per batch expanded over the queries), without the (O, rep, C)
    copy the expand would need."""
    if not 0.0 < p < 1.0:
        raise ValueError(f"dropout_bcast: p must be in (0, 1), got {p}")
    return BcastDropoutFn.apply(x.reshape(-1, x.shape[-1]), rep, p, group)


def dropout(x: torch.Tensor, p: float, training: bool, group: int = 1) -> torch.Tensor:
    """F.dropout(x, p, training) with the HIP kernel (identity when not
    training or p == 0).  Shapes the kernel cannot take (numel % 8 != 0,
    misaligned) are made contiguous and padded by the caller's layout; a
    CPU tensor raises (the product path runs on the GPU)."""
    if not training or p == 0.0:
        return x
    if not 0.0 <= p < 1.0:
        raise ValueError(f"dropout probability has to be in [0, 1), got {p}")
    if group > 1:
        return DropoutFn.apply(x, p, group)
    if x.numel() % 8 != 0:
        # tiny tensors (e.g. a (B, d) style vector with B * d % 8 != 0): flat-pad to the kernel's granule
        n = x.numel()
        flat = torch.nn.functional.pad(x.reshape(-1), (0, (-n) % 8))
        return DropoutFn.apply(flat, p)[:n].view(x.shape)
    return DropoutFn.apply(x, p)
