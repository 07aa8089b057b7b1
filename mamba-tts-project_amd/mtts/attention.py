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
from .linear import cast_scope, linear


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

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False):
        with cast_scope():
            return self._forward(query, key, value, key_padding_mask)

    def _forward(self, query, key, value, key_padding_mask):
        cd = query.dtype
        d, H = self.embed_dim, self.num_heads
        W, b = self.in_proj_weight, self.in_proj_bias
        q = linear(query, W, b, rows=(0, d))
        p_drop = self.dropout if self.training else 0.0
        if key is value:
            kv = linear(key.to(cd), W, b, rows=(d, 3 * d))
            o = attn_kernels.attention_kv(q, kv, H, key_padding_mask, p_drop)
        else:
            k = linear(key.to(cd), W, b, rows=(d, 2 * d))
            v = linear(value.to(cd), W, b, rows=(2 * d, 3 * d))
            o = attn_kernels.attention(q, k, v, H, key_padding_mask, p_drop)
        out = linear(o, self.out_proj.weight, self.out_proj.bias)
        return out, None
