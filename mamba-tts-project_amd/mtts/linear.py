"""Linear layers of the decoder hot path (projections, FFN, head).

Forward / data-gradient GEMMs of the large projections run on the
hand-written ping-pong NT MFMA kernel (csrc/gemm.hip, `proj`); skinny and
short-M ones on hipBLASLt through torch.  Further differences from nn.Linear:

* weight gradients (small output, K = B*T tokens) are computed split-K with
  fp32 partial products (4 K-chunks, summed in fp32): the stock `dy^T @ x`
  runs at 47-650 TF/s on these shapes, the split form at 140-900 TF/s, and
  the result is already the fp32 master-param gradient (no cast kernels);
* bias gradients are a HIP column sum (mtts_colsum) with fp32 accumulation.

Weights are fp32 masters.  Their compute-dtype copies are refreshed once per
top-level forward (`cast_scope`): the decoder casts every GEMM weight in ONE
HIP launch (mtts_cast_bf16_multi) into persistent buffers, writing for the
large 2-D weights a transposed bf16 copy W^T as well; nested module calls
reuse them.  The forward runs x @ W^T on W (hipBLASLt "NT"), the data
gradient dy @ W on W^T (again "NT": 1.1-1.4 PF/s on these shapes vs
0.9-1.2 for the "NN" form, tools/bench_gemm.py).  (Version counters are not
used: fused optimizers update parameters without bumping them.)
"""
from __future__ import annotations

import contextlib

import torch

from . import _lib as L
from . import gemm as G
from . import wgrad as WG

_scope = {"token": 0, "depth": 0}
_cast_plans = {}
TRANSPOSE_MIN = 512   # weights with both dims >= this also get a W^T copy


def _want_t(p):
    return p.dim() == 2 and (min(p.shape) >= TRANSPOSE_MIN or getattr(p, "_mtts_want_t", False))


def _cast_multi_bf16(params):
    """One mtts_cast_bf16_multi launch: W -> bf16 W (and W^T) for all params."""
    key = tuple((p.data_ptr(), tuple(p.shape)) for p in params)
    plan = _cast_plans.get(key)
    if plan is None:
        descs = (L.CastDesc * len(params))()
        bufs = []
        tile0 = 0
        for i, p in enumerate(params):
            ent = getattr(p, "_mtts_cast", None)
            buf = ent[1] if (ent is not None and ent[1].dtype == torch.bfloat16 and ent[1].shape == p.shape) else \
                torch.empty(p.shape, device=p.device, dtype=torch.bfloat16)
            bt = None
            if _want_t(p):
                ent = getattr(p, "_mtts_castT", None)
                tshape = (p.shape[1], p.shape[0])
                bt = ent[1] if (ent is not None and ent[1].shape == tshape) else \
                    torch.empty(tshape, device=p.device, dtype=torch.bfloat16)
            rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
            descs[i].src, descs[i].dst, descs[i].dstT = p.data_ptr(), buf.data_ptr(), L.ptr(bt)
            descs[i].rows, descs[i].cols, descs[i].tile0 = rows, cols, tile0
            tile0 += L.lib().mtts_cast_tiles(rows, cols)
            bufs.append((buf, bt))
        raw = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(params[0].device)
        plan = (raw, bufs, tile0)
        _cast_plans[key] = plan
    raw, bufs, total = plan
    L.call_raw("mtts_cast_bf16_multi", raw.data_ptr(), len(params), total)
    tok = _scope["token"]
    for p, (b, bt) in zip(params, bufs):
        p._mtts_cast = (tok, b)
        if bt is not None:
            p._mtts_castT = (tok, bt)


@contextlib.contextmanager
def cast_scope(params=None, dtype=None):
    """Open a weight-cast scope; the outermost scope invalidates all cached
    casts and (optionally) pre-casts `params` to `dtype` (bf16: one HIP
    launch, with W^T copies; otherwise one foreach copy)."""
    if _scope["depth"] == 0:
        _scope["token"] += 1
        fast = (params is not None and dtype == torch.bfloat16 and len(params) > 0 and
                all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.dim() in (1, 2)
                    for p in params))
        if fast:
            _cast_multi_bf16(list(params))
        elif params is not None and dtype is not None:
            src = [p for p in params if p.dtype != dtype and p.is_cuda]
            dst = []
            for p in src:
                ent = getattr(p, "_mtts_cast", None)
                buf = ent[1] if (ent is not None and ent[1].dtype == dtype and ent[1].shape == p.shape) else \
                    torch.empty(p.shape, device=p.device, dtype=dtype)
                dst.append(buf)
            if src:
                with torch.no_grad():
                    torch._foreach_copy_(dst, [p.detach() for p in src])
                for p, b in zip(src, dst):
                    p._mtts_cast = (_scope["token"], b)
    _scope["depth"] += 1
    try:
        yield
    finally:
        _scope["depth"] -= 1


def cast_weight(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Compute-dtype copy of a parameter, valid for the current cast scope."""
    if w.dtype == dtype:
        return w.detach()
    ent = getattr(w, "_mtts_cast", None)
    if ent is not None and ent[0] == _scope["token"] and ent[1].dtype == dtype and ent[1].device == w.device:
        return ent[1]
    if ent is not None and ent[1].dtype == dtype and ent[1].shape == w.shape:
        t = ent[1]
        with torch.no_grad():
            t.copy_(w.detach())
    else:
        t = w.detach().to(dtype)
    w._mtts_cast = (_scope["token"], t)
    return t


def cast_weight_t(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Contiguous compute-dtype W^T (cols x rows) for the current cast scope
    (made by the scope's multi-tensor cast, else transposed here)."""
    ent = getattr(w, "_mtts_castT", None)
    if ent is not None and ent[0] == _scope["token"] and ent[1].dtype == dtype:
        return ent[1]
    t = cast_weight(w, dtype).t().contiguous()
    w._mtts_castT = (_scope["token"], t)
    return t


def colsum(x2d: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """fp32 column sums of a (rows, cols) tensor with unit column stride
    (into `out`, a contiguous fp32 vector, when given)."""
    if x2d.stride(-1) != 1:
        x2d = x2d.contiguous()
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, device=x2d.device, dtype=torch.float32)
    rpg = max(rows, 1)
    wsz = L.lib().mtts_colsum_workspace(rows, cols, rpg)
    ws = torch.empty(wsz, device=x2d.device, dtype=torch.uint8) if wsz > 0 else None
    L.call_raw("mtts_colsum", x2d.data_ptr(), L.dtype_code(x2d), rows, cols, x2d.stride(0), rpg,
               out.data_ptr(), 0, L.ptr(ws))
    return out


def colsum_groups(x2d: torch.Tensor, rows_per_group: int) -> torch.Tensor:
    """fp32 column sums of each group of `rows_per_group` consecutive rows:
    (rows, cols) -> (rows / rows_per_group, cols)."""
    if x2d.stride(-1) != 1:
        x2d = x2d.contiguous()
    rows, cols = x2d.shape
    if rows % rows_per_group:
        raise ValueError(f"colsum_groups: rows={rows} not a multiple of {rows_per_group}")
    out = torch.empty(rows // rows_per_group, cols, device=x2d.device, dtype=torch.float32)
    wsz = L.lib().mtts_colsum_workspace(rows, cols, rows_per_group)
    ws = torch.empty(wsz, device=x2d.device, dtype=torch.uint8) if wsz > 0 else None
    L.call_raw("mtts_colsum", x2d.data_ptr(), L.dtype_code(x2d), rows, cols, x2d.stride(0), rows_per_group,
               out.data_ptr(), cols, L.ptr(ws))
    return out


# weight gradients with both output dims >= this run on the hand-written TN
# kernel (mtts_gemm, csrc/gemm.hip: 0.9-1.1 PF/s on the C2 shapes vs 0.6-0.83
# for the split-K bmm below); the skinny x_proj / dt_proj ones stay on it
HIP_WGRAD_MIN = 256


# forward / data-gradient projections y = x W^T (+ b) run on the hand-written
# NT kernel (mtts_gemm, ping-pong) when both weight dims are >= NT_MIN and the
# output has >= NT_MIN_TILES 256x256 tiles (half the chip): the C2 / C5
# projections (in/out_proj, attention q/out, FFN).  Skinny (x_proj, dt_proj,
# head) and short-M (text K/V, M = B * T_text) GEMMs stay on hipBLASLt, whose
# small macro-tiles fill the chip there.
NT_MIN = 256
NT_MIN_TILES = 128


def _nt_route(x2, w, bias=None):
    m, k = x2.shape
    n = w.shape[0]
    return (n >= NT_MIN and k >= NT_MIN and -(-m // G.TILE) * -(-n // G.TILE) >= NT_MIN_TILES and G.nt_ok(x2, w)
            and (bias is None or (bias.dtype in (torch.float32, torch.bfloat16) and bias.stride(-1) == 1
                                  and G.epi_ok(bias))))


def proj(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor = None) -> torch.Tensor:
    """x2 (M, K) @ w (N, K)^T (+ bias) in x2's dtype: the NT MFMA kernel when
    the shape routes there, else torch (hipBLASLt)."""
    if _nt_route(x2, w, bias):
        return G.mm_nt(x2, w, bias=bias)
    return torch.addmm(bias, x2, w.t()) if bias is not None else x2 @ w.t()


def wgrad(dy: torch.Tensor, x: torch.Tensor, splits: int = 4, out: torch.Tensor = None) -> torch.Tensor:
    """dW = dy^T @ x in fp32; dy (M, n), x (M, k) with the same dtype.
    `out` (n, k) fp32, possibly a row slice of a larger gradient, receives it."""
    M = dy.shape[0]
    if dy.dtype == torch.float32:
        return torch.mm(dy.t(), x, out=out) if out is not None else dy.t() @ x
    big = dy.shape[1] >= HIP_WGRAD_MIN and x.shape[1] >= HIP_WGRAD_MIN
    skinny = G.WGRAD_SKINNY_ON_TN and min(dy.shape[1], x.shape[1]) >= 64 and max(dy.shape[1], x.shape[1]) >= HIP_WGRAD_MIN
    out_ok = out is None or (out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0)
    if (big or skinny) and G.tn_ok(dy, x) and out_ok:
        return G.mm_tn(dy, x, out=out)
    M64 = M // 64 * 64
    if (big or skinny) and M64 >= 1024 and M != M64 and out_ok and G.tn_ok(dy[:M64], x[:M64]):
        # a ragged token count (the style frames, B * T_frame): the < 64 rows
        # past the last whole K-step by torch, then the 64-row-aligned bulk
        # accumulated on the TN kernel (beta = 1)
        tail = torch.mm(dy[M64:].t(), x[M64:], out_dtype=torch.float32)
        if out is None:
            out = tail
        else:
            out.copy_(tail)
        return G.mm_tn(dy[:M64], x[:M64], out=out, beta=1.0)
    if splits > 1 and M % splits == 0 and M >= 2048:
        m = M // splits
        part = torch.bmm(dy.reshape(splits, m, -1).transpose(1, 2), x.reshape(splits, m, -1),
                         out_dtype=torch.float32)
        return torch.sum(part, 0, out=out) if out is not None else part.sum(0)
    r = torch.mm(dy.t(), x, out_dtype=torch.float32)
    if out is not None:
        out.copy_(r)
        return out
    return r


class BiasGradSlot:
    """Hand-off of a bias gradient computed by a downstream kernel: the
    LayerNorm backward that consumes a linear layer's output (and nothing else
    does) sums its dx columns in the same pass (ops.LayerNormFn colsum_slot),
    so the linear's backward skips its own column-sum launches."""
    __slots__ = ("value",)

    def __init__(self):
        self.value = None

    def take(self, n):
        v, self.value = self.value, None
        return v if (v is not None and v.numel() == n) else None


class LinearFn(torch.autograd.Function):
    """y = x @ weight[r0:r1]^T + bias[r0:r1] in dtype of x.  Gradients for the
    full weight/bias (zero outside [r0, r1) when a row slice is used)."""

    @staticmethod
    def forward(ctx, x, weight, bias, r0, r1, slot=None, partner=None):
        cd = x.dtype
        ctx.slot = slot
        ctx.partner = partner
        w = cast_weight(weight, cd)
        if r0 is not None:
            w = w[r0:r1]
        x2 = x.reshape(-1, x.shape[-1])
        b = None
        if bias is not None:
            b = cast_weight(bias, cd)
            if r0 is not None:
                b = b[r0:r1]
        y = proj(x2, w, b)
        ctx.save_for_backward(x2, w)
        ctx.weight = weight
        ctx.meta = (x.shape, weight.shape, weight.dtype, None if bias is None else bias.dtype, r0, r1)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        xshape, wshape, wdt, bdt, r0, r1 = ctx.meta
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            if w.dtype == torch.bfloat16 and _want_t(ctx.weight):
                wt = cast_weight_t(ctx.weight, w.dtype)        # (k, n): dy @ (W^T)^T, the fast operand layout
                if r0 is not None:
                    wt = wt[:, r0:r1]
                dx = proj(dy2, wt).view(xshape)
            else:
                dx = (dy2 @ w).view(xshape)
        dW = db = None
        rest = ctx.partner.take() if ctx.partner is not None else None
        if rest is not None and r0 is not None:
            # this projection also owns the parameter's other rows (rest: the
            # layer's K/V rows of in_proj, attention.KVAllFn): ONE submit and
            # ONE bias tensor for the whole parameter -- no zero fills, copies
            # or autograd adds, and the weight gradient stays in this layer's
            # grouped launch
            dyr, xr, (q0, q1) = rest
            if ctx.needs_input_grad[1] and not WG.submit([(dy2, x2, ctx.weight, (r0, r1)),
                                                          (dyr, xr, ctx.weight, (q0, q1))]):
                dW = torch.empty(wshape, device=dy2.device, dtype=torch.float32)
                wgrad(dy2, x2, out=dW[r0:r1])
                wgrad(dyr.contiguous(), xr, out=dW[q0:q1])
                if r1 - r0 + q1 - q0 < wshape[0]:
                    for a, b in ((0, min(r0, q0)), (max(r1, q1), wshape[0])):
                        if b > a:
                            dW[a:b].zero_()
                dW = dW.to(wdt)
            if bdt is not None and ctx.needs_input_grad[2]:
                db = torch.empty(wshape[0], device=dy2.device, dtype=torch.float32)
                colsum(dy2, out=db[r0:r1])
                colsum(dyr, out=db[q0:q1])
                if r1 - r0 + q1 - q0 < wshape[0]:
                    for a, b in ((0, min(r0, q0)), (max(r1, q1), wshape[0])):
                        if b > a:
                            db[a:b].zero_()
                db = db.to(bdt)
            return dx, dW, db, None, None, None, None
        if ctx.needs_input_grad[1] and not WG.submit([(dy2, x2, ctx.weight, None if r0 is None else (r0, r1))]):
            g = wgrad(dy2, x2).to(wdt)
            if r0 is not None:
                full = torch.zeros(wshape, device=g.device, dtype=wdt)
                full[r0:r1] = g
                g = full
            dW = g
        if bdt is not None and ctx.needs_input_grad[2]:
            gb = ctx.slot.take(dy2.shape[1]) if ctx.slot is not None else None
            gb = (gb if gb is not None else colsum(dy2)).to(bdt)
            if r0 is not None:
                full = torch.zeros(wshape[0], device=gb.device, dtype=bdt)
                full[r0:r1] = gb
                gb = full
            db = gb
        return dx, dW, db, None, None, None, None


def linear(x, weight, bias=None, rows=None, dbias_slot=None, partner=None):
    """Functional form; `rows=(r0, r1)` selects a row slice of weight/bias;
    `dbias_slot` (BiasGradSlot): the bias gradient arrives from the consumer's
    backward (the caller guarantees the output feeds only that consumer);
    `partner.take()` -> (dy, x, (q0, q1)) or None: the gradient operands of
    the same parameter's other rows, whose weight / bias gradients this
    backward then produces together with its own."""
    r0, r1 = (None, None) if rows is None else rows
    return LinearFn.apply(x, weight, bias, r0, r1, dbias_slot, partner)


class FFNFn(torch.autograd.Function):
    """ff(h) = dropout_p(gelu(h W1^T + b1)) W2^T + b2 (mamba_decoder.py:39-43,
    88 with p = 0; the style blocks' nn.Sequential(Linear, GELU, Dropout,
    Linear), style_cross_attention.py:103-109, 249-255) with bf16 compute on
    the hand-written GEMM: bias + exact GELU fused into the first
    projection's epilogue (the bf16 pre-activation is written beside the
    activation for the backward), the GELU backward fused into the second
    projection's data-gradient epilogue -- or, with dropout, into the HIP
    dropout kernel that regenerates the mask (mtts.dropout) -- both weight
    gradients on the TN kernel straight into fp32."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, slot=None, p=0.0):
        from . import dropout as DO
        cd = h.dtype
        ctx.slot = slot
        W1, B1, W2, B2 = cast_weight(w1, cd), cast_weight(b1, cd), cast_weight(w2, cd), cast_weight(b2, cd)
        h2 = h.reshape(-1, h.shape[-1])
        pre = torch.empty(h2.shape[0], W1.shape[0], device=h.device, dtype=cd)
        a = G.mm_nt(h2, W1, bias=B1, gelu_aux=pre)
        ctx.p, ctx.seed = p, None
        if p > 0.0:
            ctx.seed = DO.new_seed()
            base, ctx.used = DO._slot(a)
            a = DO.apply_mask(a, p, ctx.seed, seed_in=base, seed_out=ctx.used)
        y = proj(a, W2, B2)
        ctx.save_for_backward(h2, pre, a, W1, W2)
        ctx.ws = (w1, w2)
        ctx.meta = (h.shape, w1.dtype, b1.dtype, w2.dtype, b2.dtype)
        return y.view(*h.shape[:-1], W2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        h2, pre, a, W1, W2 = ctx.saved_tensors
        hshape, w1dt, b1dt, w2dt, b2dt = ctx.meta
        w1, w2 = ctx.ws
        dy2 = dy.reshape(-1, dy.shape[-1]).to(W2.dtype)
        # d(pre) = (dy W2) * gelu'(pre), one GEMM (W2^T copy: k-contiguous operand);
        # with dropout: the dropout kernel applies the mask and gelu'(pre)
        W2t = cast_weight_t(w2, W2.dtype) if _want_t(w2) else W2.t().contiguous()
        if ctx.p > 0.0:
            from . import dropout as DO
            dpre = DO.apply_mask(G.mm_nt(dy2, W2t), ctx.p, ctx.seed, pre=pre, seed_in=ctx.used)
        else:
            dpre = G.mm_nt(dy2, W2t, dgelu_aux=pre)
        dh = None
        if ctx.needs_input_grad[0]:
            if _want_t(w1):
                dh = proj(dpre, cast_weight_t(w1, W1.dtype))
            else:
                dh = dpre @ W1
            dh = dh.view(hshape)
        dW1 = dW2 = None   # both straight to the grouped engine when deferral is on (mtts.wgrad)
        if ctx.needs_input_grad[1] and not WG.submit([(dpre, h2, w1, None)]):
            dW1 = wgrad(dpre, h2).to(w1dt)
        db1 = colsum(dpre).to(b1dt) if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[3] and not WG.submit([(dy2, a, w2, None)]):
            dW2 = wgrad(dy2, a).to(w2dt)
        db2 = None
        if ctx.needs_input_grad[4]:
            db2 = ctx.slot.take(dy2.shape[1]) if ctx.slot is not None else None
            db2 = (db2 if db2 is not None else colsum(dy2)).to(b2dt)
        return dh, dW1, db1, dW2, db2, None, None


def ffn(h, w1, b1, w2, b2, dbias_slot=None, p=0.0):
    """dropout_p(gelu(h W1^T + b1)) W2^T + b2: the fused bf16 path when the
    shapes allow it (bf16 activations, d_model / d_ff multiples of 64, rows a
    multiple of 8 when p > 0), else the per-op path (LinearFn + F.gelu + the
    HIP dropout).  dbias_slot: see linear()."""
    if (G.ENABLED and G.FFN_FUSED and h.dtype == torch.bfloat16 and h.is_cuda and h.shape[-1] % 64 == 0 and w1.shape[0] % 64 == 0
            and h.stride(-1) == 1 and h.is_contiguous()):
        return FFNFn.apply(h, w1, b1, w2, b2, dbias_slot, p)
    from . import dropout as DO
    a = DO.dropout(torch.nn.functional.gelu(linear(h, w1, b1)), p, p > 0.0)
    return linear(a, w2, b2, dbias_slot=dbias_slot)
