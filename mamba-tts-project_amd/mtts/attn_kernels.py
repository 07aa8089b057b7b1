"""Multi-head attention core o = softmax(q k^T / sqrt(hd) + mask) v.

q (B, T, H*hd), k/v (B, S, H*hd) channel-last (head-major inside the row, as
nn.MultiheadAttention's projections produce).  key_padding_mask (B, S) bool,
True = ignore.  Fully masked rows produce NaN (PyTorch MHA semantics).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def attention(q, k, v, n_heads, key_padding_mask=None, dropout_p=0.0):
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
