"""Cross-attention module with nn.MultiheadAttention's parameter layout.

Replaces nn.MultiheadAttention(embed_dim, num_heads, batch_first=True) as used
at mamba_decoder.py:32-36,72-77 and style_cross_attention.py:91-96,237-242
(query != key/value path, no attention dropout when p = 0).  state_dict keys
are identical: in_proj_weight (3d, d), in_proj_bias (3d), out_proj.{weight,bias}.

Semantics kept on purpose: key_padding_mask True =
ignore; a row whose keys are all masked yields NaN, as PyTorch MHA does.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import attn_kernels
from . import wgrad as WG
from .linear import _want_t, cast_scope, cast_weight, cast_weight_t, colsum, linear, proj, wgrad


class InProjFn(torch.autograd.Function):
    """q = query W[:d]^T + b[:d] and kv = key W[d:]^T + b[d:] (key is value):
    the packed in-projection of nn.MultiheadAttention
    (F.multi_head_attention_forward's _in_projection_packed).  The backward
    writes the full (3d, d) weight / (3d) bias gradients in place, slice by
    slice (no zero-padded per-slice gradients to add up)."""

    @staticmethod
    def forward(ctx, query, key, weight, bias):
        cd = query.dtype
        d = query.shape[-1]
        Wc, bc = cast_weight(weight, cd), cast_weight(bias, cd)
        x2, k2 = query.reshape(-1, d), key.reshape(-1, d)
        q = proj(x2, Wc[:d], bc[:d])
        kv = proj(k2, Wc[d:], bc[d:])
        ctx.save_for_backward(x2, k2, Wc)
        ctx.weight = weight
        ctx.meta = (query.shape, key.shape, weight.dtype, bias.dtype)
        return q.view(*query.shape[:-1], d), kv.view(*key.shape[:-1], 2 * d)

    @staticmethod
    def backward(ctx, dq, dkv):
        x2, k2, Wc = ctx.saved_tensors
        qshape, kshape, wdt, bdt = ctx.meta
        d = x2.shape[1]
        dq2 = dq.reshape(-1, d).to(Wc.dtype)
        dkv2 = dkv.reshape(-1, 2 * d).to(Wc.dtype)
        if Wc.dtype == torch.bfloat16 and _want_t(ctx.weight):
            Wt = cast_weight_t(ctx.weight, Wc.dtype)       # (d, 3d): dgrads as dy @ (W^T)^T
            dquery = proj(dq2, Wt[:, :d]).view(qshape) if ctx.needs_input_grad[0] else None
            dkey = proj(dkv2, Wt[:, d:]).view(kshape) if ctx.needs_input_grad[1] else None
        else:
            dquery = (dq2 @ Wc[:d]).view(qshape) if ctx.needs_input_grad[0] else None
            dkey = (dkv2 @ Wc[d:]).view(kshape) if ctx.needs_input_grad[1] else None
        dW = db = None
        if ctx.needs_input_grad[2] and not WG.submit([(dq2, x2, ctx.weight, (0, d)),
                                                      (dkv2, k2, ctx.weight, (d, 3 * d))]):
            dW = torch.empty(3 * d, d, device=x2.device, dtype=torch.float32)
            wgrad(dq2, x2, out=dW[:d])
            wgrad(dkv2, k2, out=dW[d:])
            dW = dW.to(wdt)
        if ctx.needs_input_grad[3]:
            db = torch.empty(3 * d, device=x2.device, dtype=torch.float32)
            colsum(dq2, out=db[:d])
            colsum(dkv2, out=db[d:])
            db = db.to(bdt)
        return dquery, dkey, dW, db


class CrossAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, batch_first=True, bias=True, device=None, dtype=None):
        super().__init__()
        if not batch_first:
            raise ValueError("only batch_first=True is supported (reference usage)")
        fk = {"device": device, "dtype": dtype}
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout = dropout
        self.batch_first = True
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim, **fk))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim, **fk))
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=True, **fk)
        # nn.MultiheadAttention._reset_parameters
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.constant_(self.in_proj_bias, 0.0)
        nn.init.constant_(self.out_proj.bias, 0.0)

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, _dbias_slot=None):
        """`_dbias_slot` (internal, linear.BiasGradSlot): out_proj's bias
        gradient is delivered by the consumer of the output (the decoder
        layer's fused residual + LayerNorm backward)."""
        with cast_scope():
            return self._forward(query, key, value, key_padding_mask, _dbias_slot)

    def _forward(self, query, key, value, key_padding_mask, dbias_slot=None):
        cd = query.dtype
        d, H = self.embed_dim, self.num_heads
        W, b = self.in_proj_weight, self.in_proj_bias
        p_drop = self.dropout if self.training else 0.0
        if key.shape[1] == 1 and key_padding_mask is None:
            return self._single_key(query, key, value, p_drop), None
        if key is value:
            q, kv = InProjFn.apply(query, key.to(cd), W, b)
            o = attn_kernels.attention_kv(q, kv, H, key_padding_mask, p_drop)
        else:
            q = linear(query, W, b, rows=(0, d))
            k = linear(key.to(cd), W, b, rows=(d, 2 * d))
            v = linear(value.to(cd), W, b, rows=(2 * d, 3 * d))
            o = attn_kernels.attention(q, k, v, H, key_padding_mask, p_drop)
        out = linear(o, self.out_proj.weight, self.out_proj.bias, dbias_slot=dbias_slot)
        return out, None

    def _single_key(self, query, key, value, p_drop=0.0):
        """One unmasked key (the style token of style_cross_attention.py:125-131,
        270-276): softmax over a single logit is exactly 1, so every query
        row's attention output is the value projection of that key -- out_proj(v),
        independent of q and k.  Without attention dropout only the value
        projection and out_proj run, on B rows instead of B*Tq.  With it
        (training, p > 0) each (batch, head, query) weight 1 is kept with
        probability 1 - p and scaled by 1 / (1 - p), as nn.MultiheadAttention's
        dropout on the (B, H, Tq, 1) weights: the head's slice of v is masked
        by ONE draw per (batch, query, head) (the HIP dropout, group = head
        dim), then out_proj runs on the B*Tq rows.  torch's MHA gives the q/k
        in-projection rows exactly zero gradient here (dS = P*(dP -
        rowsum(P*dP)) = 0 for one key); LinearFn's row slice reproduces that for
        the weights, and the zero-weighted key term keeps a (zero) gradient
        flowing to `key` so optimizer state and weight decay of the key path
        behave as with torch MHA."""
        cd = query.dtype
        d = self.embed_dim
        B, Tq = query.shape[0], query.shape[1]
        v = linear(value.to(cd), self.in_proj_weight, self.in_proj_bias, rows=(2 * d, 3 * d))   # (B, 1, d)
        if p_drop > 0.0:
            from . import dropout as DO
            o = DO.dropout(v.expand(B, Tq, d).contiguous(), p_drop, True, group=self.head_dim)
            o = linear(o, self.out_proj.weight, self.out_proj.bias)
            return o + 0.0 * key.to(cd).sum(dim=-1, keepdim=True)
        o = linear(v, self.out_proj.weight, self.out_proj.bias)
        o = o + 0.0 * key.to(cd).sum(dim=-1, keepdim=True)
        return o.expand(B, Tq, d).contiguous()
