"""Multi-head attention core o = softmax(q k^T / sqrt(hd) + mask) v on the HIP
kernels of libmtts (mtts_attention_fwd / _bwd, csrc/attn.hip).

q (B, T, H*hd), k/v (B, S, H*hd) channel-last (head-major inside the row, as
nn.MultiheadAttention's projections produce; reference call sites
mamba_decoder.py:72-77, style_cross_attention.py:125-131,270-276).
key_padding_mask (B, S) bool, True = ignore.  Fully masked rows produce NaN
(PyTorch MHA semantics).

Attention-weight dropout (only the style pipeline's training mode uses it,
style_cross_attention.py:91-96) has no HIP kernel: that case runs torch's
scaled_dot_product_attention, whose RNG stream no reimplementation could
match anyway.  Everything else runs on libmtts, and there is no CPU path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib as L

_HEAD_DIMS = (16, 32, 64, 128)


def _aligned(t):
    es = t.element_size()
    return (t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and (t.stride(0) * es) % 16 == 0
            and (t.stride(1) * es) % 16 == 0)


def _prep(t):
    return t if _aligned(t) else t.contiguous()


def _fwd_args(q, k, v, n_heads, kpm, out, lse):
    B, T, d = q.shape
    a = L.AttnFwdArgs()
    a.batch, a.heads, a.head_dim, a.q_len, a.kv_len = B, n_heads, d // n_heads, T, k.shape[1]
    a.dtype = L.dtype_code(q)
    a.scale = 1.0 / math.sqrt(d // n_heads)
    a.q_bs, a.q_ls = q.stride(0), q.stride(1)
    a.k_bs, a.k_ls = k.stride(0), k.stride(1)
    a.v_bs, a.v_ls = v.stride(0), v.stride(1)
    a.o_bs, a.o_ls = out.stride(0), out.stride(1)
    a.mask_bs = 0 if kpm is None else kpm.stride(0)
    a.q, a.k, a.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    a.key_padding_mask = L.ptr(kpm)
    a.out = out.data_ptr()
    a.lse = L.ptr(lse)
    return a


def _mask_u8(kpm, B, S):
    if kpm is None:
        return None
    if kpm.shape != (B, S):
        raise ValueError(f"key_padding_mask must be (B, S) = {(B, S)}, got {tuple(kpm.shape)}")
    if kpm.dtype != torch.bool:
        raise TypeError("key_padding_mask must be bool (True = ignore)")
    kpm = kpm.contiguous()
    return kpm.view(torch.uint8)


def attention_decode_packed(q, k, v, n_heads, kpm=None):
    """Single-query attention (q (B, d), decode step) returning the output
    as the packed activation image of the output projection (ops.PackedAct;
    csrc/attn.hip single-pass decode kernel).  k / v: (B, S, d) channel-last,
    or HEAD-MAJOR (B, H, S, hd) contiguous (the decode engine's per-context
    copies): one contiguous K and V block per (batch, head)."""
    from .ops import PackedAct
    B, d = q.shape
    q3 = q[:, None]
    if not _aligned(q3):
        q3 = q3.contiguous()
    if k.dim() == 4:   # head-major
        H, S, hd = k.shape[1:]
        if H != n_heads or H * hd != d or not (k.is_contiguous() and v.is_contiguous()):
            raise ValueError("attention_decode_packed: head-major k / v must be contiguous (B, H, S, hd)")
        m = _mask_u8(kpm, B, S)
        out = torch.empty(B, 1, d, device=q.device, dtype=q.dtype)
        yp = PackedAct.empty(B, d, q.device)
        a = _fwd_args(q3, k.view(B, H * S, hd), v.view(B, H * S, hd), n_heads, m, out, None)
        a.kv_len, a.k_ls, a.v_ls, a.kv_hs = S, hd, hd, S * hd
        a.out_packed = yp.data.data_ptr()
        L.call("mtts_attention_fwd", a)
        return yp
    k, v = _prep(k), _prep(v)
    m = _mask_u8(kpm, B, k.shape[1])
    out = torch.empty(B, 1, d, device=q.device, dtype=q.dtype)
    yp = PackedAct.empty(B, d, q.device)
    a = _fwd_args(q3, k, v, n_heads, m, out, None)
    a.out_packed = yp.data.data_ptr()
    L.call("mtts_attention_fwd", a)
    return yp


def attention_decode_qproj_packed(x, wq, bq, ln_w, ln_b, eps, k, v, n_heads, kpm=None):
    """Single-query cross-attention with the query projection fused in
    (mtts_attention_decode_qproj): q = bf16(LN(x) wq^T + bq) per (batch,
    head) inside the decode kernel, LN(x) = bf16(LayerNorm(x) * ln_w + ln_b)
    as the packed projections' LayerNorm prologue computes it; k / v
    head-major (B, H, S, hd) contiguous.  Returns the output as the packed
    activation image of the output projection (ops.PackedAct)."""
    from .ops import PackedAct
    B, d = x.shape
    if k.dim() != 4 or not (k.is_contiguous() and v.is_contiguous()):
        raise ValueError("attention_decode_qproj_packed: head-major contiguous (B, H, S, hd) k / v")
    if x.dtype != torch.bfloat16 or x.stride(1) != 1 or wq.dtype != torch.bfloat16 or wq.stride(1) != 1 \
            or wq.stride(0) != d:
        raise ValueError("attention_decode_qproj_packed: bf16 x (B, d) and row-major bf16 wq (d, d)")
    H, S, hd = k.shape[1:]
    m = _mask_u8(kpm, B, S)
    yp = PackedAct.empty(B, d, x.device)
    q3 = x[:, None]
    a = _fwd_args(q3, k.view(B, H * S, hd), v.view(B, H * S, hd), n_heads, m, q3, None)   # no row-major out
    a.kv_len, a.k_ls, a.v_ls, a.kv_hs = S, hd, hd, S * hd
    a.out = 0
    a.out_packed = yp.data.data_ptr()
    qa = L.AttnQProjArgs()
    qa.f = a
    qa.x, qa.x_rs = x.data_ptr(), x.stride(0)
    qa.wq, qa.bq = wq.data_ptr(), L.ptr(bq)
    lw, lb = ln_w.detach().float().contiguous(), ln_b.detach().float().contiguous()
    qa.ln_w, qa.ln_b, qa.eps, qa.d_model = lw.data_ptr(), lb.data_ptr(), float(eps), d
    L.call("mtts_attention_decode_qproj", qa)
    return yp


def attention_fwd(q, k, v, n_heads, kpm=None, want_lse=False):
    """Returns (out (B, T, d) in q's dtype, lse (B, H, T) fp32 or None)."""
    for t in (q, k, v):
        if not t.is_cuda:
            raise RuntimeError("libmtts ops need CUDA (HIP) tensors; there is no CPU path")
    B, T, d = q.shape
    if d % n_heads or (d // n_heads) not in _HEAD_DIMS:
        raise ValueError(f"head_dim {d}/{n_heads} not supported (need one of {_HEAD_DIMS})")
    if not (q.dtype == k.dtype == v.dtype):
        raise TypeError("q, k, v must share a dtype")
    q, k, v = _prep(q), _prep(k), _prep(v)
    m = _mask_u8(kpm, B, k.shape[1])
    out = torch.empty(B, T, d, device=q.device, dtype=q.dtype)
    lse = torch.empty(B, n_heads, T, device=q.device, dtype=torch.float32) if want_lse else None
    L.call("mtts_attention_fwd", _fwd_args(q, k, v, n_heads, m, out, lse))
    return out, lse


def attention_bwd(q, k, v, n_heads, kpm, out, lse, dout, dk=None, dv=None, dq=None):
    """Returns (dq, dk, dv); dq/dk/dv may be given as (strided) output views."""
    B, T, d = q.shape
    S = k.shape[1]
    dout = _prep(dout.to(q.dtype))
    m = _mask_u8(kpm, B, S)
    if dq is None:
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
    if dk is None:
        dk = torch.empty(B, S, d, device=q.device, dtype=q.dtype)
    if dv is None:
        dv = torch.empty(B, S, d, device=q.device, dtype=q.dtype)
    a = L.AttnBwdArgs()
    a.f = _fwd_args(q, k, v, n_heads, m, out, lse)
    a.dout, a.do_bs, a.do_ls = dout.data_ptr(), dout.stride(0), dout.stride(1)
    a.dq, a.dq_bs, a.dq_ls = dq.data_ptr(), dq.stride(0), dq.stride(1)
    a.dk, a.dk_bs, a.dk_ls = dk.data_ptr(), dk.stride(0), dk.stride(1)
    a.dv, a.dv_bs, a.dv_ls = dv.data_ptr(), dv.stride(0), dv.stride(1)
    ws_bytes = L.lib().mtts_attention_bwd_workspace(B, n_heads, d // n_heads, T, S, L.dtype_code(q))
    ws = torch.empty(ws_bytes, device=q.device, dtype=torch.uint8)
    a.workspace = ws.data_ptr()
    L.call("mtts_attention_bwd", a)
    return dq, dk, dv


class AttentionFn(torch.autograd.Function):
    """Separate k / v inputs."""

    @staticmethod
    def forward(ctx, q, k, v, n_heads, kpm):
        q, k, v = _prep(q), _prep(k), _prep(v)
        out, lse = attention_fwd(q, k, v, n_heads, kpm, want_lse=True)
        ctx.save_for_backward(q, k, v, out, lse, kpm)
        ctx.n_heads = n_heads
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse, kpm = ctx.saved_tensors
        dq, dk, dv = attention_bwd(q, k, v, ctx.n_heads, kpm, out, lse, dout)
        return dq, dk, dv, None, None


class AttentionKVFn(torch.autograd.Function):
    """k = kv[..., :d], v = kv[..., d:] of one projection output: the gradient
    is written straight into one (B, S, 2d) tensor (no slice-backward copies)."""

    @staticmethod
    def forward(ctx, q, kv, n_heads, kpm):
        d = q.shape[-1]
        q = _prep(q)
        # the K/V gradient's destination when kv is a column view of the
        # layers' batched K/V projection (attention.KVAllFn / DkvSink)
        ctx.sink = getattr(kv, "_mtts_dkv_sink", None)
        if not _aligned(kv[..., :d]) or not _aligned(kv[..., d:]):
            kv = kv.contiguous()
        out, lse = attention_fwd(q, kv[..., :d], kv[..., d:], n_heads, kpm, want_lse=True)
        ctx.save_for_backward(q, kv, out, lse, kpm)
        ctx.n_heads = n_heads
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, out, lse, kpm = ctx.saved_tensors
        d = q.shape[-1]
        dkv = None
        if ctx.sink is not None:
            sink, layer = ctx.sink
            dkv = sink.view(layer)
            if dkv.shape != kv.shape or not (_aligned(dkv[..., :d]) and _aligned(dkv[..., d:])):
                dkv = None
        if dkv is None:
            dkv = torch.empty(kv.shape, device=kv.device, dtype=kv.dtype)
        dq, _, _ = attention_bwd(q, kv[..., :d], kv[..., d:], ctx.n_heads, kpm, out, lse, dout,
                                 dk=dkv[..., :d], dv=dkv[..., d:])
        return dq, dkv, None, None


class AttentionQKVFn(torch.autograd.Function):
    """Self-attention on one fused projection output qkv (B, T, 3d): q, k, v
    are its thirds and the gradient is written straight into one (B, T, 3d)
    tensor (no slice-backward copies or adds)."""

    @staticmethod
    def forward(ctx, qkv, n_heads, kpm):
        d = qkv.shape[-1] // 3
        if not all(_aligned(qkv[..., i * d:(i + 1) * d]) for i in range(3)):
            qkv = qkv.contiguous()
        q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
        out, lse = attention_fwd(q, k, v, n_heads, kpm, want_lse=True)
        ctx.save_for_backward(qkv, out, lse, kpm)
        ctx.n_heads = n_heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, kpm = ctx.saved_tensors
        d = qkv.shape[-1] // 3
        dqkv = torch.empty(qkv.shape, device=qkv.device, dtype=qkv.dtype)
        attention_bwd(qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:], ctx.n_heads, kpm, out, lse, dout,
                      dq=dqkv[..., :d], dk=dqkv[..., d:2 * d], dv=dqkv[..., 2 * d:])
        return dqkv, None, None


def attention_qkv(qkv, n_heads, key_padding_mask=None, dropout_p=0.0):
    """Self-attention of q, k, v = the thirds of qkv (B, T, 3d)."""
    d = qkv.shape[-1] // 3
    if dropout_p > 0.0:
        return _sdpa_dropout(qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:], n_heads, key_padding_mask, dropout_p)
    if torch.is_grad_enabled() and qkv.requires_grad:
        return AttentionQKVFn.apply(qkv, n_heads, key_padding_mask)
    return attention_fwd(qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:], n_heads, key_padding_mask)[0]


def _sdpa_dropout(q, k, v, n_heads, key_padding_mask, dropout_p):
    B, T, d = q.shape
    S = k.shape[1]
    hd = d // n_heads
    qh = q.view(B, T, n_heads, hd).transpose(1, 2)
    kh = k.reshape(B, S, n_heads, hd).transpose(1, 2)
    vh = v.reshape(B, S, n_heads, hd).transpose(1, 2)
    mask = None
    if key_padding_mask is not None:
        mask = torch.zeros(B, 1, 1, S, device=q.device, dtype=q.dtype)
        mask = mask.masked_fill(key_padding_mask[:, None, None, :], float("-inf"))
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask, dropout_p=dropout_p)
    return o.transpose(1, 2).reshape(B, T, d)


def attention(q, k, v, n_heads, key_padding_mask=None, dropout_p=0.0):
    if dropout_p > 0.0:
        return _sdpa_dropout(q, k, v, n_heads, key_padding_mask, dropout_p)
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        return AttentionFn.apply(q, k, v, n_heads, key_padding_mask)
    return attention_fwd(q, k, v, n_heads, key_padding_mask)[0]


def attention_kv(q, kv, n_heads, key_padding_mask=None, dropout_p=0.0):
    d = q.shape[-1]
    if dropout_p > 0.0:
        return _sdpa_dropout(q, kv[..., :d], kv[..., d:], n_heads, key_padding_mask, dropout_p)
    if torch.is_grad_enabled() and (q.requires_grad or kv.requires_grad):
        return AttentionKVFn.apply(q, kv, n_heads, key_padding_mask)
    return attention_fwd(q, kv[..., :d], kv[..., d:], n_heads, key_padding_mask)[0]
