"""Codec-token cross-entropy on libmtts (csrc/loss.hip).

Reference: train.py:31-42 `codec_ce_loss` = F.cross_entropy(logits.view(B*T,
V), targets.view(B*T), ignore_index=pad_id): mean over the non-ignored rows
(NaN when every target is ignored, as torch).  Forward and backward are one
HIP launch pair each, fp32 math, deterministic; bf16 logits are read as
they are (no fp32 copy) and get bf16 gradients.  No CPU path.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


def _args(logits, targets, ignore_index, loss, lse, ws):
    a = L.CrossEntropyArgs()
    a.rows, a.vocab, a.dtype, a.ld = logits.shape[0], logits.shape[1], L.dtype_code(logits), logits.stride(0)
    a.logits, a.targets, a.ignore_index = logits.data_ptr(), targets.data_ptr(), int(ignore_index)
    a.loss, a.lse, a.workspace = loss.data_ptr(), lse.data_ptr(), ws.data_ptr()
    return a


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        if not logits.is_cuda:
            raise RuntimeError("libmtts ops need CUDA (HIP) tensors; there is no CPU path")
        if logits.dim() != 2 or logits.stride(1) != 1 or logits.dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("cross_entropy: logits must be (rows, V) fp32 / bf16 with unit column stride")
        targets = targets.reshape(-1).to(torch.int64).contiguous()
        if targets.numel() != logits.shape[0]:
            raise ValueError("cross_entropy: one target per row")
        rows = logits.shape[0]
        dev = logits.device
        loss = torch.empty(2, device=dev, dtype=torch.float32)
        lse = torch.empty(rows, device=dev, dtype=torch.float32)
        ws = torch.empty(L.lib().mtts_cross_entropy_workspace(rows) // 4, device=dev, dtype=torch.float32)
        a = _args(logits, targets, ignore_index, loss, lse, ws)
        L.call("mtts_cross_entropy_fwd", a)
        ctx.save_for_backward(logits, targets, loss, lse)
        ctx.ignore_index = ignore_index
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        logits, targets, loss, lse = ctx.saved_tensors
        dl = torch.empty(logits.shape, device=logits.device, dtype=logits.dtype)
        a = _args(logits, targets, ctx.ignore_index, loss, lse, lse)
        g = g.reshape(1).to(torch.float32).contiguous()
        L.call_raw("mtts_cross_entropy_bwd", C.byref(a), C.c_void_p(g.data_ptr()), C.c_void_p(dl.data_ptr()),
                   C.c_int64(dl.stride(0)))
        return dl, None, None


def cross_entropy(logits, targets, ignore_index=-100):
    """F.cross_entropy(logits, targets, ignore_index=...) with mean reduction,
    for (rows, V) logits (fp32 or bf16; the reference's `.float()` upcast is
    done in registers)."""
    return CrossEntropyFn.apply(logits, targets, ignore_index)
