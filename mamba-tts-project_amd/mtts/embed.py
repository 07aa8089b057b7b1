"""Embedding sums of the decoder: the token + quantizer + position prologue of
MambaTTSDecoder.forward (reference mamba_decoder.py:167-171) and the
reference-voice embedding of the training loop (train.py:115-131,
embed_codec_tokens), as one autograd function over one HIP kernel.

Forward: mtts_embed_sum, one wave per output row, out[b, l] =
tok_w[tokens[b, l]] + q_w[qid[l]] + pos_w[pid[l]] (fp32 tables, fp32 sum,
output in the compute dtype); qid / pid are per-position int32 ids shared by
the batch.  The backward is what matters: nn.Embedding's dense backward
sorts the 16k indices of a batch and scatters (~0.55 ms per C2 step for the
three tables, dominated by a 10-entry codec vocabulary every row collides
on).  Here, with S = sum over the batch of dy (L, d) in fp32:
  * position table: pid = arange(L) -> d_pos[:L] = S; pid = arange(T).repeat(Q)
    -> d_pos[:T] = sum of S's Q blocks; otherwise index_add_;
  * quantizer table (<= 64 rows): onehot(qid)^T @ S;
  * token table (<= 16 rows, the codec vocabulary): mtts_embed_table_grad, one
    HIP pass over dy with the vocabulary's bins in registers (the one-hot GEMM
    it replaces ran ~91 us per C5 call on hipBLASLt); up to 64 rows
    onehot(ids)^T @ dy; larger tables: index_add_ (atomic scatter).
All parameter gradients are fp32 (the master dtype).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib as L

SMALL_VOCAB = 64
HIP_VOCAB = 16      # mtts_embed_table_grad's register bins
_err = {}


def _table_grad(ids2d, g2d, rows):
    ids = ids2d.reshape(-1)
    if (rows <= HIP_VOCAB and ids.dtype == torch.int64 and g2d.dtype in (torch.float32, torch.bfloat16)
            and g2d.stride(-1) == 1 and g2d.stride(0) % 8 == 0 and g2d.shape[1] % 8 == 0
            and g2d.data_ptr() % 16 == 0):
        ids = ids.contiguous()
        n, d = g2d.shape
        out = torch.empty(rows, d, device=g2d.device, dtype=torch.float32)
        ws = torch.empty(L.lib().mtts_embed_table_grad_workspace(n, d, rows), device=g2d.device, dtype=torch.uint8)
        L.call_raw("mtts_embed_table_grad", ids.data_ptr(), n, g2d.data_ptr(), L.dtype_code(g2d), g2d.stride(0), d,
                   rows, out.data_ptr(), ws.data_ptr())
        return out
    if rows <= SMALL_VOCAB:
        oh = F.one_hot(ids2d.reshape(-1), rows).to(g2d.dtype)
        if g2d.dtype == torch.float32:
            return oh.t() @ g2d
        return torch.mm(oh.t(), g2d, out_dtype=torch.float32)
    out = torch.zeros(rows, g2d.shape[1], device=g2d.device, dtype=torch.float32)
    out.index_add_(0, ids2d.reshape(-1), g2d.float())
    return out


def _err_flag(dev):
    f = _err.get(dev)
    if f is None:
        f = torch.zeros(1, device=dev, dtype=torch.int32)
        _err[dev] = f
    return f


def check_errors():
    """Raise if any mtts_embed_sum launch saw a token id outside its table
    (nn.Embedding raises there; the kernel only flags it, without a host sync)."""
    for dev, f in _err.items():
        if int(f.item()):
            f.zero_()
            raise IndexError(f"embedding: token id out of range (device {dev})")


class EmbedSumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, qid, pid, tok_w, q_w, pos_w, out_dtype, pos_repeat):
        B, Ln = tokens.shape
        d = tok_w.shape[1]
        tw, qw, pw = (w.detach().float().contiguous() for w in (tok_w, q_w, pos_w))
        tk = tokens if tokens.stride(-1) == 1 else tokens.contiguous()
        out = torch.empty(B, Ln, d, device=tokens.device, dtype=out_dtype)
        L.call_raw("mtts_embed_sum", tk.data_ptr(), tk.stride(0), qid.data_ptr(), pid.data_ptr(), tw.data_ptr(),
                   qw.data_ptr(), pw.data_ptr(), B, Ln, d, tw.shape[0], out.data_ptr(), L.dtype_code(out),
                   out.stride(0), _err_flag(tokens.device).data_ptr())
        ctx.save_for_backward(tokens, qid, pid)
        ctx.meta = (tok_w.shape[0], q_w.shape[0], pos_w.shape[0], tok_w.dtype, q_w.dtype, pos_w.dtype, pos_repeat)
        return out

    @staticmethod
    def backward(ctx, dx):
        tokens, qid, pid = ctx.saved_tensors
        V, Qn, P, tdt, qdt, pdt, pos_repeat = ctx.meta
        B, Ln = tokens.shape
        d = dx.shape[-1]
        g2d = dx.reshape(B * Ln, d)
        d_tok = _table_grad(tokens, g2d, V).to(tdt) if ctx.needs_input_grad[3] else None
        d_q = d_pos = None
        if ctx.needs_input_grad[4] or ctx.needs_input_grad[5]:
            S = torch.sum(dx.view(B, Ln, d), 0, dtype=torch.float32)        # (L, d)
            if ctx.needs_input_grad[4]:
                d_q = (F.one_hot(qid.long(), Qn).float().t() @ S if Qn <= SMALL_VOCAB else
                       torch.zeros(Qn, d, device=dx.device).index_add_(0, qid.long(), S)).to(qdt)
            if ctx.needs_input_grad[5]:
                d_pos = torch.zeros(P, d, device=dx.device, dtype=torch.float32)
                if pos_repeat == 1:                                          # pid = arange(L)
                    d_pos[:Ln] = S
                elif pos_repeat > 1:                                         # pid = arange(T).repeat(Q)
                    T = Ln // pos_repeat
                    d_pos[:T] = S.view(pos_repeat, T, d).sum(0)
                else:
                    d_pos.index_add_(0, pid.long(), S)
                d_pos = d_pos.to(pdt)
        return None, None, None, d_tok, d_q, d_pos, None, None


def _ids(n, dev, fill=None, values=None):
    if values is not None:
        return values.to(device=dev, dtype=torch.int32).contiguous()
    return torch.full((n,), fill, device=dev, dtype=torch.int32) if fill is not None else \
        torch.arange(n, device=dev, dtype=torch.int32)


def embed_sum(tokens, quant_ids, tok_w, q_w, pos_w, out_dtype):
    """Decoder prologue: tokens (B, L); quant_ids (L,) or (B, L) with equal
    rows (batch-shared); positions 0..L-1."""
    dev = tokens.device
    Ln = tokens.shape[1]
    q = quant_ids[0] if quant_ids.dim() == 2 else quant_ids
    return EmbedSumFn.apply(tokens, _ids(Ln, dev, values=q), _ids(Ln, dev), tok_w, q_w, pos_w, out_dtype, 1)


def embed_codec_layout(tokens_3d, tok_w, q_w, pos_w, out_dtype):
    """train.py:115-131 layout: tokens (B, Q, T) flattened quantizer-major to
    (B, Q*T); quantizer id q and position t for element (q, t)."""
    B, Q, T = tokens_3d.shape
    dev = tokens_3d.device
    flat = tokens_3d.reshape(B, Q * T)
    qid = torch.arange(Q, device=dev, dtype=torch.int32).repeat_interleave(T)
    pid = torch.arange(T, device=dev, dtype=torch.int32).repeat(Q)
    return EmbedSumFn.apply(flat, qid, pid, tok_w, q_w, pos_w, out_dtype, Q)
