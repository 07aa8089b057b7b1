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


class DkvSink:
    """One (M, L*2d) buffer for the K/V gradients of the L layers whose K/V
    projections ran as one GEMM (KVAllFn): each layer's attention backward
    writes its dK / dV straight into its column slice, so the projection's
    backward reads them as ONE operand (no per-layer copies or adds)."""

    def __init__(self, rows, n_layers, width, shape, device, dtype):
        self.rows, self.L, self.width, self.shape = rows, n_layers, width, shape
        self.device, self.dtype = device, dtype
        self.buf = None
        self.key2 = None                   # the (M, d) key rows the projections read (set by KVAllFn)
        self.written = [False] * n_layers  # the layer's dK / dV landed (attention backward)
        self.taken = [False] * n_layers    # its weight / bias gradients were produced by the q projection

    def view(self, layer):
        if self.buf is None:
            self.buf = torch.empty(self.rows, self.L * self.width, device=self.device, dtype=self.dtype)
        self.written[layer] = True
        return self.buf[:, layer * self.width:(layer + 1) * self.width].view(*self.shape, self.width)

    def partner(self, layer):
        """For the layer's q projection (linear(..., partner=)): hands over the
        layer's K/V gradient rows d:3d of in_proj once its attention backward
        has written them."""
        sink = self

        class _P:
            @staticmethod
            def take():
                if not sink.written[layer] or sink.buf is None or sink.key2 is None:
                    return None
                sink.taken[layer] = True
                d = sink.width // 2
                return (sink.buf[:, layer * sink.width:(layer + 1) * sink.width], sink.key2, (d, 3 * d))
        return _P()


class KVAllFn(torch.autograd.Function):
    """kv_l = key W_l[d:]^T + b_l[d:] for every decoder layer l at once: the
    layers' cross-attention K/V in-projections (nn.MultiheadAttention's
    packed in_proj, mamba_decoder.py:72-77) all read the SAME text (+ voice
    prompt) hidden states, so they run as ONE (M, L*2d) NT GEMM over the
    stacked weight rows instead of L short-M GEMMs (C2: M = B*T_text = 1024,
    twelve 1024 x 2048 x 1024 products).  The outputs are column views of
    that product; the backward takes the L K/V gradients as one operand (the
    attention backward writes them into a DkvSink) for ONE key gradient GEMM
    (K = L*2d: the sum over layers inside the reduction, no autograd adds of
    L (B, T_kv, d) gradients).  Each layer's K/V weight / bias gradient rows
    d:3d are produced by that layer's q projection together with its own rows
    0:d (LinearFn `partner`): one submit to the grouped engine per layer (in
    that layer's launch), one bias tensor, no zero fills or adds."""

    @staticmethod
    def forward(ctx, key, sink, *params):
        cd = key.dtype
        d = key.shape[-1]
        Ws, bs = params[0::2], params[1::2]
        k2 = key.reshape(-1, d)
        Wst = torch.cat([cast_weight(W, cd)[d:] for W in Ws])             # (L*2d, d)
        bst = torch.cat([cast_weight(b, cd)[d:] for b in bs])
        kv = proj(k2, Wst, bst)                                           # (M, L*2d)
        ctx.save_for_backward(k2)
        ctx.Ws, ctx.bs, ctx.kshape, ctx.sink = Ws, bs, key.shape, sink
        sink.key2 = k2
        return tuple(kv[:, l * 2 * d:(l + 1) * 2 * d].view(*key.shape[:-1], 2 * d) for l in range(len(Ws)))

    @staticmethod
    def backward(ctx, *dkvs):
        (k2,) = ctx.saved_tensors
        Ws, bs, sink = ctx.Ws, ctx.bs, ctx.sink
        nl, d = len(Ws), k2.shape[1]
        w2 = 2 * d
        cd = k2.dtype
        in_sink = sink.buf is not None and all(
            g is not None and g.data_ptr() == sink.buf.data_ptr() + l * w2 * sink.buf.element_size()
            and g.stride()[-2] == nl * w2 for l, g in enumerate(dkvs))
        if in_sink:
            dkv = sink.buf
        else:   # a layer's gradient arrived elsewhere (unused layer, accumulated use): assemble
            dkv = torch.zeros(k2.shape[0], nl * w2, device=k2.device, dtype=cd)
            for l, g in enumerate(dkvs):
                if g is not None:
                    dkv[:, l * w2:(l + 1) * w2] = g.reshape(-1, w2)
        sink.buf = None
        dkey = None
        if ctx.needs_input_grad[0]:
            if cd == torch.bfloat16:
                WstT = torch.cat([cast_weight_t(W, cd)[:, d:] for W in Ws], dim=1)   # (d, L*2d)
                dkey = proj(dkv, WstT).view(ctx.kshape)
            else:
                dkey = (dkv @ torch.cat([cast_weight(W, cd)[d:] for W in Ws])).view(ctx.kshape)
        grads = [dkey, None]
        # the layers' weight / bias gradients were produced by each layer's q
        # projection (LinearFn partner); only a layer whose q projection did
        # not take them is handled here
        for l in range(nl):
            W, b = Ws[l], bs[l]
            dW = db = None
            if not sink.taken[l]:
                dy = dkv[:, l * w2:(l + 1) * w2]
                if ctx.needs_input_grad[2 + 2 * l] and not WG.submit([(dy, k2, W, (d, 3 * d))]):
                    dW = torch.zeros(W.shape, device=W.device, dtype=W.dtype)
                    dW[d:] = wgrad(dy.contiguous(), k2).to(W.dtype)
                if ctx.needs_input_grad[3 + 2 * l]:
                    db = torch.zeros(b.shape, device=b.device, dtype=b.dtype)
                    db[d:] = colsum(dy).to(b.dtype)
            grads += [dW, db]
        # ready for another backward through the same graph (retain_graph)
        sink.written = [False] * nl
        sink.taken = [False] * nl
        return tuple(grads)


def kv_all(key: torch.Tensor, attns) -> list:
    """The K/V in-projections of `attns` (CrossAttention modules of equal
    width, packed in_proj with bias) over one shared `key`, as KVAllFn; a
    list of (B, T_kv, 2d) column views, one per module."""
    params = []
    for a in attns:
        params += [a.in_proj_weight, a.in_proj_bias]
    d = attns[0].embed_dim
    sink = DkvSink(key.numel() // d, len(attns), 2 * d, tuple(key.shape[:-1]), key.device, key.dtype)
    outs = list(KVAllFn.apply(key, sink, *params))
    for l, o in enumerate(outs):
        o._mtts_dkv_sink = (sink, l)     # read by the attention backward (attn_kernels.AttentionKVFn)
    return outs


def kv_all_ok(key: torch.Tensor, attns) -> bool:
    a0 = attns[0]
    d = a0.embed_dim
    return (len(attns) >= 2 and key.dim() == 3 and key.shape[-1] == d and key.shape[1] > 1 and key.is_cuda
            and all(a.embed_dim == d and a.in_proj_bias is not None and a.in_proj_weight.dtype == torch.float32
                    and a.in_proj_bias.dtype == torch.float32 and a.in_proj_weight.is_contiguous()
                    and a.dropout == 0.0 for a in attns))


class _KeyTie(torch.autograd.Function):
    """Returns `o` unchanged and gives `key` an exactly-zero gradient (torch
    MHA's gradient to a single key: dS = P * (dP - rowsum(P * dP)) = 0), so
    optimizer state / weight decay of the key path behave as with torch MHA,
    without a (B, Tq, d) broadcast add in the forward and its reduction over
    Tq in the backward (what `o + 0 * key.sum()` would cost)."""

    @staticmethod
    def forward(ctx, o, key):
        ctx.kmeta = (key.shape, key.dtype, key.device)
        return o.view_as(o)

    @staticmethod
    def backward(ctx, do):
        shape, dt, dev = ctx.kmeta
        return do, torch.zeros(shape, dtype=dt, device=dev)


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

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, _dbias_slot=None, _kv=None):
        """`_dbias_slot` (internal, linear.BiasGradSlot): out_proj's bias
        gradient is delivered by the consumer of the output (the decoder
        layer's fused residual + LayerNorm backward).  `_kv` (internal): this
        module's K/V projection of `key` (= `value`), computed with other
        layers' by `kv_all`."""
        with cast_scope():
            return self._forward(query, key, value, key_padding_mask, _dbias_slot, _kv)

    def _forward(self, query, key, value, key_padding_mask, dbias_slot=None, kv_pre=None):
        cd = query.dtype
        d, H = self.embed_dim, self.num_heads
        W, b = self.in_proj_weight, self.in_proj_bias
        p_drop = self.dropout if self.training else 0.0
        if kv_pre is not None:
            sk = getattr(kv_pre, "_mtts_dkv_sink", None)
            q = linear(query, W, b, rows=(0, d), partner=None if sk is None else sk[0].partner(sk[1]))
            o = attn_kernels.attention_kv(q, kv_pre, H, key_padding_mask, p_drop)
            return linear(o, self.out_proj.weight, self.out_proj.bias, dbias_slot=dbias_slot), None
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
            # the value row broadcast over the queries and dropped in one HIP pass
            o = DO.dropout_bcast(v.reshape(B, d), Tq, p_drop, group=self.head_dim)
            o = linear(o, self.out_proj.weight, self.out_proj.bias)
        else:
            o = linear(v, self.out_proj.weight, self.out_proj.bias).expand(B, Tq, d).contiguous()
        return _KeyTie.apply(o, key) if torch.is_grad_enabled() and key.requires_grad else o
