"""Token + quantizer + position embedding sum of MambaTTSDecoder.forward
(reference mamba_decoder.py:201-206: token_embed(audio) + pos_embed(pos) +
quant_embed(quant_ids)) as one autograd function.

Forward is three gathers and an add (HBM-bound, torch ops).  The backward is
what matters: nn.Embedding's dense backward sorts the 16k indices of a batch
and scatters (≈0.55 ms per C2 step for the three tables, dominated by a
10-entry codec vocabulary that every row collides on).  Here:
  * position table: rows 0..T-1, d_pos[t] = sum_b dy[b, t]  (one reduction);
  * small tables (<= 64 rows, e.g. codec ids, quantizer ids):
    d_W = onehot(ids)^T @ dy, one skinny GEMM reading dy once;
  * larger tables: index_add_ (atomic scatter).
All parameter gradients are fp32 (the master dtype).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

SMALL_VOCAB = 64


def _table_grad(ids2d, g2d, rows):
    if rows <= SMALL_VOCAB:
        oh = F.one_hot(ids2d.reshape(-1), rows).to(g2d.dtype)
        if g2d.dtype == torch.float32:
            return oh.t() @ g2d
        return torch.mm(oh.t(), g2d, out_dtype=torch.float32)
    out = torch.zeros(rows, g2d.shape[1], device=g2d.device, dtype=torch.float32)
    out.index_add_(0, ids2d.reshape(-1), g2d.float())
    return out


class EmbedSumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, quant_ids, tok_w, q_w, pos_w, out_dtype):
        B, T = tokens.shape
        pos = pos_w[:T]
        x = F.embedding(tokens, tok_w) + F.embedding(quant_ids, q_w) + pos[None]
        ctx.save_for_backward(tokens, quant_ids)
        ctx.meta = (tok_w.shape[0], q_w.shape[0], pos_w.shape[0], tok_w.dtype, q_w.dtype, pos_w.dtype)
        return x.to(out_dtype)

    @staticmethod
    def backward(ctx, dx):
        tokens, quant_ids = ctx.saved_tensors
        V, Qn, P, tdt, qdt, pdt = ctx.meta
        B, T = tokens.shape
        d = dx.shape[-1]
        g2d = dx.reshape(B * T, d)
        d_tok = _table_grad(tokens, g2d, V).to(tdt) if ctx.needs_input_grad[2] else None
        d_q = _table_grad(quant_ids, g2d, Qn).to(qdt) if ctx.needs_input_grad[3] else None
        d_pos = None
        if ctx.needs_input_grad[4]:
            d_pos = torch.empty(P, d, device=dx.device, dtype=torch.float32)
            torch.sum(dx.view(B, T, d), 0, dtype=torch.float32, out=d_pos[:T])
            d_pos[T:].zero_()
            d_pos = d_pos.to(pdt)
        return None, None, d_tok, d_q, d_pos, None


def embed_sum(tokens, quant_ids, tok_w, q_w, pos_w, out_dtype):
    return EmbedSumFn.apply(tokens, quant_ids, tok_w, q_w, pos_w, out_dtype)
