"""Tensor-level wrappers and autograd Functions over libmtts.so.

Every function here launches HIP kernels through the C ABI (mtts._lib); none
falls back to PyTorch arithmetic.  Activations are channel-last (B, L, C).

Public op API mirroring [upstream] mamba-ssm (layout (B, D, L)):
    selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                      delta_softplus=False, return_last_state=False)
    causal_conv1d_fn(x, weight, bias=None, activation=None)
    causal_conv1d_update(x, conv_state, weight, bias=None, activation=None)
    selective_state_update(state, x, dt, A, B, C, D=None, z=None,
                           dt_bias=None, dt_softplus=False)
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L

SCAN_CKPT = 16  # must equal kSub in scan.hip


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("libmtts ops need CUDA (HIP) tensors; there is no CPU path")


def _f32c(t):
    return None if t is None else t.detach().to(torch.float32).contiguous()


def _bc_ok(t):
    """B/C views must have N-stride 1 and 16-byte aligned rows."""
    es = t.element_size()
    return (t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and (t.stride(0) * es) % 16 == 0
            and (t.stride(1) * es) % 16 == 0)


def _bc(t):
    return t if _bc_ok(t) else t.contiguous()


# ---------------------------------------------------------------------------
# selective scan (channel-last)
# ---------------------------------------------------------------------------
def _scan_args(u, delta, A, Bm, Cm, D, z, delta_bias, softplus, h0, out, last, ckpt, a_is_log=False):
    Bsz, Ln, Dm = u.shape
    for t in (u, delta, out) + ((z,) if z is not None else ()):
        if t.stride(-1) != 1:
            raise ValueError("scan: channel stride must be 1")
    a = L.ScanFwdArgs()
    a.batch, a.seqlen, a.dim, a.dstate = Bsz, Ln, Dm, A.shape[1]
    a.dtype_io, a.dtype_bc = L.dtype_code(u), L.dtype_code(Bm)
    a.delta_softplus = int(bool(softplus))
    a.ckpt_chunk = SCAN_CKPT if ckpt is not None else 0
    a.a_is_log = int(bool(a_is_log))
    a.u_bs, a.u_ls = u.stride(0), u.stride(1)
    a.delta_bs, a.delta_ls = delta.stride(0), delta.stride(1)
    if z is not None:
        a.z_bs, a.z_ls = z.stride(0), z.stride(1)
    a.out_bs, a.out_ls = out.stride(0), out.stride(1)
    a.B_bs, a.B_ls = Bm.stride(0), Bm.stride(1)
    a.C_bs, a.C_ls = Cm.stride(0), Cm.stride(1)
    a.u, a.delta, a.A, a.Bm, a.Cm = u.data_ptr(), delta.data_ptr(), A.data_ptr(), Bm.data_ptr(), Cm.data_ptr()
    a.D, a.z, a.delta_bias, a.h0 = L.ptr(D), L.ptr(z), L.ptr(delta_bias), L.ptr(h0)
    a.out, a.last_state, a.ckpt = out.data_ptr(), L.ptr(last), L.ptr(ckpt)
    return a


def scan_fwd(u, delta, A, Bm, Cm, D=None, z=None, delta_bias=None, softplus=True, h0=None,
             want_last=False, want_ckpt=False, out=None, a_is_log=False):
    """u, delta, z: (B, L, D) channel-last; Bm, Cm: (B, L, N); A: (D, N) fp32
    (a_is_log: A holds A_log, the kernels use -exp(A_log)).
    Returns (out, last_state | None, ckpt | None)."""
    _check_cuda(u, delta, A, Bm, Cm, D, z, delta_bias, h0)
    Bsz, Ln, Dm = u.shape
    N = A.shape[1]
    if delta.dtype != u.dtype or (z is not None and z.dtype != u.dtype):
        raise TypeError("scan: u/delta/z must share a dtype")
    Bm, Cm = _bc(Bm), _bc(Cm)
    if Cm.dtype != Bm.dtype:
        Cm = Cm.to(Bm.dtype)
    A, D, delta_bias, h0 = _f32c(A), _f32c(D), _f32c(delta_bias), _f32c(h0)
    if out is None:
        out = torch.empty(Bsz, Ln, Dm, device=u.device, dtype=u.dtype)
    last = torch.empty(Bsz, Dm, N, device=u.device, dtype=torch.float32) if want_last else None
    ckpt = (torch.empty(Bsz, (Ln + SCAN_CKPT - 1) // SCAN_CKPT, Dm, N, device=u.device, dtype=torch.float32)
            if want_ckpt else None)
    a = _scan_args(u, delta, A, Bm, Cm, D, z, delta_bias, softplus, h0, out, last, ckpt, a_is_log)
    wsz = L.lib().mtts_selective_scan_fwd_workspace(Bsz, Dm, Ln, N)
    ws = torch.empty(wsz, device=u.device, dtype=torch.uint8) if wsz > 0 else None
    a.workspace = L.ptr(ws)
    L.call("mtts_selective_scan_fwd", a)
    return out, last, ckpt


def scan_bwd(u, delta, A, Bm, Cm, D, z, delta_bias, softplus, h0, ckpt, dout,
             du=None, ddelta=None, dz=None, dB=None, dC=None, need_dh0=False, a_is_log=False, workspace=None):
    """Backward of scan_fwd.  du/ddelta/dz may be preallocated (strided)
    views to write into; dB/dC (B, L, N) fp32 views likewise.
    Returns du, ddelta, dz, dB, dC, dA, dD, ddelta_bias, dh0 (with a_is_log
    the returned dA is the gradient w.r.t. A_log)."""
    Bsz, Ln, Dm = u.shape
    N = A.shape[1]
    dev = u.device
    Bm, Cm = _bc(Bm), _bc(Cm)
    if Cm.dtype != Bm.dtype:
        Cm = Cm.to(Bm.dtype)
    A, D, delta_bias, h0 = _f32c(A), _f32c(D), _f32c(delta_bias), _f32c(h0)
    dout = dout if dout.stride(-1) == 1 else dout.contiguous()
    if dout.dtype != u.dtype:
        dout = dout.to(u.dtype)
    du = torch.empty(Bsz, Ln, Dm, device=dev, dtype=u.dtype) if du is None else du
    ddelta = torch.empty(Bsz, Ln, Dm, device=dev, dtype=u.dtype) if ddelta is None else ddelta
    if z is not None and dz is None:
        dz = torch.empty(Bsz, Ln, Dm, device=dev, dtype=u.dtype)
    dB = torch.empty(Bsz, Ln, N, device=dev, dtype=torch.float32) if dB is None else dB
    dC = torch.empty(Bsz, Ln, N, device=dev, dtype=torch.float32) if dC is None else dC
    dA = torch.empty(Dm, N, device=dev, dtype=torch.float32)
    dD = torch.empty(Dm, device=dev, dtype=torch.float32)
    dbias = torch.empty(Dm, device=dev, dtype=torch.float32)
    dh0 = torch.empty(Bsz, Dm, N, device=dev, dtype=torch.float32) if need_dh0 else None
    ws = workspace if workspace is not None else \
        torch.empty(L.lib().mtts_selective_scan_bwd_workspace(Bsz, Dm, Ln, N), device=dev, dtype=torch.uint8)
    dummy_out = dout  # the forward's `out` is not read by the backward
    b = L.ScanBwdArgs()
    b.f = _scan_args(u, delta, A, Bm, Cm, D, z, delta_bias, softplus, h0, dummy_out, None, ckpt, a_is_log)
    b.dout, b.dout_bs, b.dout_ls = dout.data_ptr(), dout.stride(0), dout.stride(1)
    b.du, b.du_bs, b.du_ls = du.data_ptr(), du.stride(0), du.stride(1)
    b.ddelta, b.ddelta_bs, b.ddelta_ls = ddelta.data_ptr(), ddelta.stride(0), ddelta.stride(1)
    if dz is not None:
        b.dz, b.dz_bs, b.dz_ls = dz.data_ptr(), dz.stride(0), dz.stride(1)
    b.dB, b.dB_bs, b.dB_ls = dB.data_ptr(), dB.stride(0), dB.stride(1)
    b.dC, b.dC_bs, b.dC_ls = dC.data_ptr(), dC.stride(0), dC.stride(1)
    b.dA, b.dD, b.ddelta_bias, b.dh0, b.workspace = dA.data_ptr(), dD.data_ptr(), dbias.data_ptr(), L.ptr(dh0), ws.data_ptr()
    L.call("mtts_selective_scan_bwd", b)
    return du, ddelta, dz, dB, dC, dA, dD, dbias, dh0


class SelectiveScanFn(torch.autograd.Function):
    """Channel-last selective scan with autograd (fwd + bwd in HIP)."""

    @staticmethod
    def forward(ctx, u, delta, A, Bm, Cm, D, z, delta_bias, softplus, return_last_state):
        out, last, ckpt = scan_fwd(u, delta, A, Bm, Cm, D, z, delta_bias, softplus, want_last=True, want_ckpt=True)
        ctx.softplus = softplus
        ctx.has = (D is not None, z is not None, delta_bias is not None)
        ctx.bc_dtype = Bm.dtype
        ctx.save_for_backward(u, delta, A, Bm, Cm, D, z, delta_bias, ckpt)
        ctx.mark_non_differentiable(last)
        return out, last

    @staticmethod
    def backward(ctx, dout, dlast):
        u, delta, A, Bm, Cm, D, z, delta_bias, ckpt = ctx.saved_tensors
        du, ddelta, dz, dB, dC, dA, dD, dbias, _ = scan_bwd(u, delta, A, Bm, Cm, D, z, delta_bias, ctx.softplus,
                                                            None, ckpt, dout)
        hasD, hasz, hasb = ctx.has
        return (du, ddelta, dA.to(A.dtype), dB.to(Bm.dtype), dC.to(Cm.dtype), dD.to(D.dtype) if hasD else None,
                dz if hasz else None, dbias.to(delta_bias.dtype) if hasb else None, None, None)


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """mamba-ssm signature and (B, D, L) layout; see oracle selective_scan_ref."""
    cl = lambda t: None if t is None else t.transpose(1, 2).contiguous()  # noqa: E731
    out, last = SelectiveScanFn.apply(cl(u), cl(delta), A, cl(B), cl(C), D, cl(z), delta_bias, delta_softplus,
                                      return_last_state)
    out = out.transpose(1, 2)
    return (out, last) if return_last_state else out


# ---------------------------------------------------------------------------
# causal conv1d (channel-last)
# ---------------------------------------------------------------------------
def _conv_args(x, w, bias, silu, state_in, out, state_out):
    Bsz, Ln, Dm = x.shape
    a = L.ConvFwdArgs()
    a.batch, a.dim, a.seqlen, a.width, a.dtype, a.silu = Bsz, Dm, Ln, w.shape[-1], L.dtype_code(x), int(silu)
    a.x_bs, a.x_ls = x.stride(0), x.stride(1)
    a.out_bs, a.out_ls = out.stride(0), out.stride(1)
    a.x, a.w, a.bias, a.conv_state_in = x.data_ptr(), w.data_ptr(), L.ptr(bias), L.ptr(state_in)
    a.out, a.conv_state_out = out.data_ptr(), L.ptr(state_out)
    return a


def conv_fwd(x, w, bias=None, silu=True, state_in=None, want_state=False, out=None):
    """x (B, L, D) channel-last (may be a strided view); w (D, K)."""
    _check_cuda(x, w, bias, state_in)
    if x.stride(-1) != 1:
        x = x.contiguous()
    Bsz, Ln, Dm = x.shape
    w = _f32c(w.reshape(Dm, -1))
    bias, state_in = _f32c(bias), _f32c(state_in)
    out = torch.empty(Bsz, Ln, Dm, device=x.device, dtype=x.dtype) if out is None else out
    st = torch.empty(Bsz, Dm, w.shape[1], device=x.device, dtype=torch.float32) if want_state else None
    L.call("mtts_causal_conv1d_fwd", _conv_args(x, w, bias, silu, state_in, out, st))
    return out, st


def conv_bwd(x, w, bias, dout, silu=True, dx=None, state_in=None):
    """Backward of conv_fwd: dx (into `dx` if given), dw, db.  `state_in`
    (B, D, K) is the forward's left history (recomputed pre-activations and
    dw include it); its own gradient is not produced here."""
    Bsz, Ln, Dm = x.shape
    w = _f32c(w.reshape(Dm, -1))
    bias, state_in = _f32c(bias), _f32c(state_in)
    dout = dout if dout.stride(-1) == 1 else dout.contiguous()
    if dout.dtype != x.dtype:
        dout = dout.to(x.dtype)
    dx = torch.empty(Bsz, Ln, Dm, device=x.device, dtype=x.dtype) if dx is None else dx
    dw = torch.empty(Dm, w.shape[1], device=x.device, dtype=torch.float32)
    db = torch.empty(Dm, device=x.device, dtype=torch.float32)
    ws = torch.empty(L.lib().mtts_causal_conv1d_bwd_workspace(Bsz, Dm, Ln, w.shape[1]), device=x.device,
                     dtype=torch.uint8)
    b = L.ConvBwdArgs()
    b.f = _conv_args(x, w, bias, silu, state_in, dout, None)
    b.dout, b.dout_bs, b.dout_ls = dout.data_ptr(), dout.stride(0), dout.stride(1)
    b.dx, b.dx_bs, b.dx_ls = dx.data_ptr(), dx.stride(0), dx.stride(1)
    b.dw, b.dbias, b.workspace = dw.data_ptr(), db.data_ptr(), ws.data_ptr()
    L.call("mtts_causal_conv1d_bwd", b)
    return dx, dw, db


class CausalConv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, silu):
        out, _ = conv_fwd(x, w, bias, silu)
        ctx.silu = silu
        ctx.save_for_backward(x, w, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, bias = ctx.saved_tensors
        if x.stride(-1) != 1:
            x = x.contiguous()
        dx, dw, db = conv_bwd(x, w, bias, dout, ctx.silu)
        return dx, dw.reshape(w.shape).to(w.dtype), (db.to(bias.dtype) if bias is not None else None), None


def causal_conv1d_fn(x, weight, bias=None, activation=None):
    """[upstream] causal_conv1d_fn signature, x (B, D, L)."""
    silu = activation in ("silu", "swish")
    out = CausalConv1dFn.apply(x.transpose(1, 2), weight, bias, silu)
    return out.transpose(1, 2)


# ---------------------------------------------------------------------------
# decode step
# ---------------------------------------------------------------------------
def conv_update(x, conv_state, w, bias=None, silu=True, out=None):
    """x (B, D); conv_state (B, D, K) fp32 updated IN PLACE.  Returns out (B, D)."""
    _check_cuda(x, conv_state, w)
    Bsz, Dm = x.shape
    if x.stride(-1) != 1:
        x = x.contiguous()
    out = torch.empty(Bsz, Dm, device=x.device, dtype=x.dtype) if out is None else out
    a = L.ConvUpdateArgs()
    a.batch, a.dim, a.width, a.dtype, a.silu = Bsz, Dm, conv_state.shape[-1], L.dtype_code(x), int(silu)
    a.x_bs, a.out_bs = x.stride(0), out.stride(0)
    a.x, a.conv_state, a.w, a.bias, a.out = x.data_ptr(), conv_state.data_ptr(), w.data_ptr(), L.ptr(bias), out.data_ptr()
    L.call("mtts_causal_conv1d_update", a)
    return out


def state_update(state, x, dt, A, Bm, Cm, D=None, z=None, dt_bias=None, softplus=True, out=None, dt_w=None,
                 packed_out=False):
    """state (B, D, N) fp32 updated IN PLACE; x/z (B, D); Bm/Cm (B, N) with
    unit element stride; dt (B, D) raw delta, or with dt_w (D, R) given the
    (B, R) low-rank input of dt_proj (fused: delta = dt @ dt_w.t()).
    packed_out: y is returned ONLY as a PackedAct (out_proj's operand)."""
    _check_cuda(state, x, dt, A, Bm, Cm, dt_w)
    for t in (Bm, Cm, dt):
        if t.stride(-1) != 1:
            raise ValueError("state_update: B / C / dt need unit element stride")
    Bsz, Dm = x.shape
    yp = PackedAct.empty(Bsz, Dm, x.device) if packed_out else None
    if not packed_out:
        out = torch.empty(Bsz, Dm, device=x.device, dtype=x.dtype) if out is None else out
    a = L.StateUpdateArgs()
    a.batch, a.dim, a.dstate = Bsz, Dm, state.shape[-1]
    a.dtype_io, a.dtype_bc, a.dt_softplus = L.dtype_code(x), L.dtype_code(Bm), int(softplus)
    a.x_bs, a.dt_bs, a.B_bs, a.C_bs = x.stride(0), dt.stride(0), Bm.stride(0), Cm.stride(0)
    a.out_bs = 0 if out is None else out.stride(0)
    if z is not None:
        a.z_bs = z.stride(0)
    a.state, a.x, a.dt, a.A, a.Bm, a.Cm = state.data_ptr(), x.data_ptr(), dt.data_ptr(), A.data_ptr(), Bm.data_ptr(), Cm.data_ptr()
    a.D, a.z, a.dt_bias, a.out = L.ptr(D), L.ptr(z), L.ptr(dt_bias), L.ptr(out)
    if yp is not None:
        a.out_packed = yp.data.data_ptr()
    if dt_w is not None:
        if dt_w.dtype != x.dtype or dt_w.shape != (Dm, dt.shape[1]) or not dt_w.is_contiguous() or dt.dtype != x.dtype:
            raise ValueError("state_update: dt_w must be a contiguous (D, R) tensor of x's dtype")
        a.dt_rank, a.dt_w = dt_w.shape[1], dt_w.data_ptr()
    L.call("mtts_selective_state_update", a)
    return out if yp is None else yp


def causal_conv1d_update(x, conv_state, weight, bias=None, activation=None):
    """[upstream] signature: x (B, D), conv_state (B, D, K) fp32 (in place)."""
    return conv_update(x, conv_state, _f32c(weight.reshape(x.shape[1], -1)), _f32c(bias),
                       activation in ("silu", "swish"))


def selective_state_update(state, x, dt, A, B, C, D=None, z=None, dt_bias=None, dt_softplus=False):
    """[upstream] signature: state (B, D, N) fp32 (in place)."""
    return state_update(state, x, dt, _f32c(A), B.contiguous(), C.contiguous(), _f32c(D), z, _f32c(dt_bias),
                        dt_softplus)


# ---------------------------------------------------------------------------
# LayerNorm (+ residual, + FiLM)
# ---------------------------------------------------------------------------
def _rows(t):
    """(..., N) with last stride 1 -> (rows, row_stride)."""
    n = t.shape[-1]
    if t.stride(-1) != 1:
        raise ValueError("layernorm: last stride must be 1")
    rows = t.numel() // n
    if t.dim() == 1:
        return rows, n
    # require a uniform row stride over the flattened leading dims
    st = t.stride(-2)
    for d in range(t.dim() - 2):
        if t.shape[d] > 1 and t.stride(d) != st * _prod(t.shape[d + 1:-1]):
            raise ValueError("layernorm: leading dims must be collapsible")
    return rows, st


def _prod(s):
    p = 1
    for v in s:
        p *= v
    return p


def _ln_args(x, w, b, eps, res, x_sum, gamma, beta, rows_per_group, y, mean, rstd):
    rows, xrs = _rows(x)
    a = L.LNArgs()
    a.rows, a.cols, a.dtype, a.eps = rows, x.shape[-1], L.dtype_code(x), float(eps)
    a.rows_per_group = int(rows_per_group) if gamma is not None else 0
    a.x_rs, a.y_rs = xrs, _rows(y)[1]
    a.x, a.w, a.b, a.y, a.mean, a.rstd = x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    if res is not None:
        a.res, a.res_rs = res.data_ptr(), _rows(res)[1]
        if x_sum is not None:
            a.x_sum, a.xsum_rs = x_sum.data_ptr(), _rows(x_sum)[1]
    if gamma is not None:
        a.gamma, a.beta, a.gb_rs, a.gb_dtype = gamma.data_ptr(), beta.data_ptr(), gamma.stride(0), L.dtype_code(gamma)
    return a


def layernorm_fwd(x, w, b, eps=1e-5, res=None, gamma=None, beta=None, rows_per_group=1, want_sum=True):
    """y = LN(x [+ res]) * w + b [then gamma*y + beta per row group].
    Returns (y, mean, rstd, x_sum | None)."""
    _check_cuda(x, w, b, res, gamma, beta)
    if x.stride(-1) != 1:
        x = x.contiguous()
    if res is not None and (res.shape != x.shape):
        raise ValueError("layernorm: res shape mismatch")
    if res is not None and res.dtype != x.dtype:
        res = res.to(x.dtype)
    w, b = _f32c(w), _f32c(b)
    if gamma is not None:
        gamma = gamma if gamma.stride(-1) == 1 else gamma.contiguous()
        beta = beta if beta.stride(-1) == 1 else beta.contiguous()
        if beta.stride(0) != gamma.stride(0):
            beta = beta.contiguous()
            gamma = gamma.contiguous()
    rows = x.numel() // x.shape[-1]
    y = torch.empty(x.shape, device=x.device, dtype=x.dtype)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    x_sum = torch.empty(x.shape, device=x.device, dtype=x.dtype) if (res is not None and want_sum) else None
    L.call("mtts_layernorm_fwd", _ln_args(x, w, b, eps, res, x_sum, gamma, beta, rows_per_group, y, mean, rstd))
    return y, mean, rstd, x_sum


def layernorm_bwd(xn, w, b, eps, gamma, beta, rows_per_group, mean, rstd, dy, dx_acc=None, dgb=None,
                  dx_colsum=None):
    """xn: the normalised input (x, or x + res).  Returns dx, dw, db, dgamma, dbeta.
    dgb: an fp32 (G, 2N) buffer receiving dgamma | dbeta side by side (then
    returned as the two halves); dx_colsum: an fp32 (N) buffer receiving the
    column sums of dx (the bias gradient of the linear that produced x)."""
    dy = dy if dy.stride(-1) == 1 else dy.contiguous()
    if dy.dtype != xn.dtype:
        dy = dy.to(xn.dtype)
    w, b = _f32c(w), _f32c(b)
    rows, cols = mean.numel(), xn.shape[-1]
    dx = torch.empty(xn.shape, device=xn.device, dtype=xn.dtype)
    dw = torch.empty(cols, device=xn.device, dtype=torch.float32)
    db = torch.empty(cols, device=xn.device, dtype=torch.float32)
    film = gamma is not None
    G = rows // rows_per_group if film else 0
    if film and dgb is not None:
        dg, dbe = dgb[:, :cols], dgb[:, cols:]
    else:
        dg = torch.empty(G, cols, device=xn.device, dtype=torch.float32) if film else None
        dbe = torch.empty(G, cols, device=xn.device, dtype=torch.float32) if film else None
    ws = torch.empty(L.lib().mtts_layernorm_bwd_workspace(rows, cols, rows_per_group if film else 0),
                     device=xn.device, dtype=torch.uint8)
    bb = L.LNBwdArgs()
    bb.f = _ln_args(xn, w, b, eps, None, None, gamma, beta, rows_per_group, xn, mean, rstd)
    bb.dy, bb.dy_rs = dy.data_ptr(), _rows(dy)[1]
    if dx_acc is not None:
        dx_acc = dx_acc if dx_acc.stride(-1) == 1 else dx_acc.contiguous()
        if dx_acc.dtype != xn.dtype:
            dx_acc = dx_acc.to(xn.dtype)
        bb.dx_acc, bb.dxacc_rs = dx_acc.data_ptr(), _rows(dx_acc)[1]
    bb.dx, bb.dx_rs = dx.data_ptr(), _rows(dx)[1]
    bb.dw, bb.db, bb.dgamma, bb.dbeta, bb.workspace = dw.data_ptr(), db.data_ptr(), L.ptr(dg), L.ptr(dbe), ws.data_ptr()
    bb.dgb_rs = dg.stride(0) if film else 0
    bb.dx_colsum = L.ptr(dx_colsum)
    L.call("mtts_layernorm_bwd", bb)
    return dx, dw, db, dg, dbe


class LayerNormFn(torch.autograd.Function):
    """y = FiLM(LN(x [+ res])); returns (y, x_sum) where x_sum = x + res (or x).
    FiLM parameters either as gamma / beta (G, N) or as ONE (G, 2N) tensor
    `film` = gamma | beta (the layout of tanh(style_mlp(z)), mamba_decoder.py
    :82-84), whose gradient is then written in place, side by side (no split /
    cat).  `colsum_slot` (a linear.BiasGradSlot): the backward also writes the
    column sums of dx into it -- the bias gradient of the linear layer whose
    output is x, when x feeds nothing but this LayerNorm."""

    @staticmethod
    def forward(ctx, x, res, w, b, gamma, beta, eps, rows_per_group, film, colsum_slot):
        if film is not None:
            n = x.shape[-1]
            gamma, beta = film[:, :n], film[:, n:]
        y, mean, rstd, x_sum = layernorm_fwd(x, w, b, eps, res, gamma, beta, rows_per_group)
        xn = x_sum if res is not None else x
        ctx.set_materialize_grads(False)   # an unused x_sum: no zero-filled gradient, no dx_acc pass
        ctx.eps, ctx.rpg = eps, rows_per_group
        ctx.has_res = res is not None
        ctx.has_film = film is not None
        ctx.slot = colsum_slot
        ctx.dtypes = (w.dtype, b.dtype, None if gamma is None else gamma.dtype)
        ctx.save_for_backward(xn, w, b, gamma, beta, mean, rstd)
        if res is None:
            x_sum = x.new_empty(0)
            ctx.mark_non_differentiable(x_sum)
        return y, x_sum

    @staticmethod
    def backward(ctx, dy, dsum):
        xn, w, b, gamma, beta, mean, rstd = ctx.saved_tensors
        if dsum is not None and dsum.numel() == 0:
            dsum = None
        if dy is None:   # only x_sum was used
            dy = torch.zeros_like(xn)
        n = xn.shape[-1]
        dgb = None
        if ctx.has_film:
            dgb = torch.empty(gamma.shape[0], 2 * n, device=xn.device, dtype=torch.float32)
        csum = None
        if ctx.slot is not None:
            csum = torch.empty(n, device=xn.device, dtype=torch.float32)
        dx, dw, db, dg, dbe = layernorm_bwd(xn, w, b, ctx.eps, gamma, beta, ctx.rpg, mean, rstd, dy, dx_acc=dsum,
                                            dgb=dgb, dx_colsum=csum)
        if csum is not None:
            ctx.slot.value = csum
        wd, bd, gd = ctx.dtypes
        dres = dx if ctx.has_res else None
        if ctx.has_film:
            return (dx, dres, dw.to(wd), db.to(bd), None, None, None, None, dgb.to(gd), None)
        return (dx, dres, dw.to(wd), db.to(bd), None if dg is None else dg.to(gd),
                None if dbe is None else dbe.to(gd), None, None, None, None)


def layer_norm(x, w, b, eps=1e-5, res=None, gamma=None, beta=None, rows_per_group=1, film=None, colsum_slot=None):
    """Returns (y, x_sum) with x_sum = x + res (an empty tensor when res is None).
    film: (G, 2N) gamma | beta in one tensor (instead of gamma / beta);
    colsum_slot: see LayerNormFn."""
    return LayerNormFn.apply(x, res, w, b, gamma, beta, eps, rows_per_group, film, colsum_slot)


# ---------------------------------------------------------------------------
# length regulator (style_cross_attention.py:156-198)
# ---------------------------------------------------------------------------

def _dur_f32(durations):
    d = durations.detach()
    if d.dtype != torch.float32:
        d = d.to(torch.float32)
    return d if d.stride(-1) == 1 else d.contiguous()


def length_regulate_lengths(durations):
    """lengths[b] = sum_t max(round(durations[b,t]), 0) as int64, on device."""
    _check_cuda(durations)
    d = _dur_f32(durations)
    B, T = d.shape
    out = torch.empty(B, device=d.device, dtype=torch.int64)
    L.call_raw("mtts_length_regulate_lengths", d.data_ptr(), d.stride(0), B, T, out.data_ptr())
    return out


class LengthRegulateFn(torch.autograd.Function):
    """out = hidden rows repeated by rounded, clamped durations, zero-padded
    to max_len; backward = per-phoneme segment sums of dout."""

    @staticmethod
    def forward(ctx, hidden, durations, max_len):
        _check_cuda(hidden, durations)
        h = hidden if hidden.stride(-1) == 1 else hidden.contiguous()
        d = _dur_f32(durations)
        B, T, D = h.shape
        out = torch.empty(B, max_len, D, device=h.device, dtype=h.dtype)
        L.call_raw("mtts_length_regulate_fwd", h.data_ptr(), L.dtype_code(h), B, T, D, h.stride(0), h.stride(1),
                   d.data_ptr(), d.stride(0), max_len, out.data_ptr(), out.stride(0), out.stride(1))
        ctx.save_for_backward(d)
        ctx.meta = (T, max_len)
        return out

    @staticmethod
    def backward(ctx, dout):
        (d,) = ctx.saved_tensors
        T, max_len = ctx.meta
        g = dout if dout.stride(-1) == 1 else dout.contiguous()
        B, _, D = g.shape
        dh = torch.empty(B, T, D, device=g.device, dtype=g.dtype)
        L.call_raw("mtts_length_regulate_bwd", g.data_ptr(), L.dtype_code(g), B, T, D, g.stride(0), g.stride(1),
                   d.data_ptr(), d.stride(0), max_len, dh.data_ptr(), dh.stride(0), dh.stride(1))
        return dh, None, None


def length_regulate(hidden, durations, max_len=None):
    """(expanded (B, max_len, D), lengths (B,) int64).  With max_len None the
    output is as long as the longest row (one device->host read, as in the
    reference's output_lengths.max().item())."""
    lengths = length_regulate_lengths(durations)
    if max_len is None:
        max_len = int(lengths.max().item()) if lengths.numel() > 0 else 0
    return LengthRegulateFn.apply(hidden, durations, int(max_len)), lengths


# ---------------------------------------------------------------------------
# decode-step projections (M <= 32 rows)
# ---------------------------------------------------------------------------
GEMM_ROWS_MAX = 32


class PackedRows:
    """A bf16 decode weight (N, K) re-laid by mtts_pack_rows_weight into
    MFMA-fragment order (csrc/gemv.hip): every weight load of the packed
    projection kernel is one coalesced KiB.  `data` is the packed image."""

    __slots__ = ("data", "N", "K", "dtype")

    def __init__(self, data, N, K):
        self.data, self.N, self.K, self.dtype = data, N, K, torch.bfloat16

    @property
    def shape(self):
        return (self.N, self.K)


class PackedAct:
    """A decode-step activation (M <= 32 rows, K columns, bf16) as the packed
    image the projection kernel loads in coalesced KiB (csrc/common.h
    xpk_index: 32 * K elements, rows >= M unused).  Made by the producers'
    epilogues (projections, state update, decode attention) and by
    ln_rows_packed."""

    __slots__ = ("data", "M", "K")

    def __init__(self, data, M, K):
        self.data, self.M, self.K = data, M, K

    @property
    def shape(self):
        return (self.M, self.K)

    @staticmethod
    def empty(M, K, device):
        if M > GEMM_ROWS_MAX or K % 32:
            raise ValueError(f"PackedAct: M={M} must be <= {GEMM_ROWS_MAX}, K={K} a multiple of 32")
        return PackedAct(torch.empty(32 * K, device=device, dtype=torch.bfloat16), M, K)

    @staticmethod
    def pack(x):
        """Packed image of a row-major bf16 (M, K) tensor (setup-time helper:
        per-context constants such as the FiLM rows)."""
        M, K = x.shape
        out = PackedAct.empty(M, K, x.device)
        img = torch.zeros(32, K, device=x.device, dtype=torch.bfloat16)
        img[:M] = x
        out.data.copy_(img.view(2, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).reshape(-1))
        return out

    def unpack(self):
        """Row-major (M, K) copy (tests / debugging)."""
        img = self.data.view(self.K // 32, 2, 4, 16, 8)            # s, half, g, r, q
        return img.permute(1, 3, 0, 2, 4).reshape(32, self.K)[:self.M]


def ln_rows_packed(x, w, b, eps, gamma=None, beta=None):
    """bf16(LN(x) * w + b [, gamma * . + beta]) of <= 32 bf16 rows as the
    packed image of the next projection (mtts_layernorm_rows_packed): the
    same values as layer_norm's y, bit for bit."""
    _check_cuda(x, w, b, gamma, beta)
    M, K = x.shape
    if x.dtype != torch.bfloat16 or x.stride(1) != 1:
        raise ValueError("ln_rows_packed: x must be bf16 (M, K) with unit column stride")
    out = PackedAct.empty(M, K, x.device)
    a = L.LNArgs()
    a.rows, a.cols, a.dtype, a.rows_per_group, a.eps = M, K, L.dtype_code(x), 1, float(eps)
    a.x, a.x_rs = x.data_ptr(), x.stride(0)
    wf, bf = _f32c(w), _f32c(b)
    a.w, a.b = wf.data_ptr(), bf.data_ptr()
    if gamma is not None:
        if gamma.dtype != torch.bfloat16 or gamma.shape != (M, K) or gamma.stride() != beta.stride() \
                or gamma.stride(1) != 1:
            raise ValueError("ln_rows_packed: FiLM gamma / beta must be (M, K) bf16 with equal strides")
        a.gamma, a.beta, a.gb_rs, a.gb_dtype = gamma.data_ptr(), beta.data_ptr(), gamma.stride(0), L.dtype_code(gamma)
    L.call_raw("mtts_layernorm_rows_packed", C.byref(a), out.data.data_ptr())
    return out


def gemv_split_ok(K, ln=False):
    """K values the packed kernel takes: K / 32 = KS * S, KS <= 8 a power
    of two, S in {1, 2, 4, 8, 16}; with the LayerNorm prologue K <= 2048
    (host mirror of gemv_split / launch_gemv_packed)."""
    if ln and K > 2048:
        return False
    if K <= 0 or K % 64:
        return False
    n, ks = K // 32, 1
    while ks < 8 and n % (2 * ks) == 0:
        ks *= 2
    return n // ks in (1, 2, 4, 8, 16)


def pack_rows_weight(w):
    """PackedRows image of a contiguous-rows bf16 weight (N, K) (one launch)."""
    _check_cuda(w)
    if w.dtype != torch.bfloat16 or w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("pack_rows_weight: weight must be 2-D bf16 with unit column stride")
    N, K = w.shape
    if not gemv_split_ok(K):
        raise ValueError(f"pack_rows_weight: K={K} unsupported by the packed kernel")
    nbytes = L.lib().mtts_pack_rows_bytes(N, K)
    out = torch.empty(nbytes // 2, device=w.device, dtype=torch.bfloat16)
    L.call_raw("mtts_pack_rows_weight", w.data_ptr(), w.stride(0), N, K, out.data_ptr())
    return PackedRows(out, N, K)


def gemm_rows_ok(x, weight):
    """True when mtts_gemm_rows_bf16 takes y = x @ weight.t() as given."""
    if isinstance(x, PackedAct):
        return isinstance(weight, PackedRows) and x.K == weight.K
    if isinstance(weight, PackedRows):
        return (x.dtype == torch.bfloat16 and x.dim() == 2 and 0 < x.shape[0] <= GEMM_ROWS_MAX
                and x.shape[1] == weight.K and x.stride(1) == 1 and x.stride(0) % 8 == 0
                and x.data_ptr() % 16 == 0)
    return (x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and x.dim() == 2
            and 0 < x.shape[0] <= GEMM_ROWS_MAX and x.shape[1] % 64 == 0 and x.stride(1) == 1
            and weight.stride(1) == 1 and x.stride(0) % 8 == 0 and weight.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0)


def gemm_rows_ln_ok(K):
    """K values the one-trip LayerNorm prologue of csrc/rows.hip takes."""
    return K in {64 * c for c in (1, 2, 4, 8)} | {128 * c for c in (1, 2, 4, 8)}


_rows_ws = {}


def rows_workspace(device):
    """Per-device split-K scratch of the decode projections: fp32 partial
    slabs and per-tile tickets (zeroed once; every launch leaves them zero).
    Allocate outside graph capture (DecodeEngine does, before capturing)."""
    key = torch.device(device)
    ws = _rows_ws.get(key)
    if ws is None:
        ws = (torch.empty(ROWS_MAX_TILES * ROWS_MAX_KG * 1024, device=key, dtype=torch.float32),
              torch.zeros(ROWS_MAX_TILES, device=key, dtype=torch.int32))
        _rows_ws[key] = ws
    return ws


ROWS_MAX_TILES, ROWS_MAX_KG = 512, 16
# Cross-workgroup split-K of the decode projections: built, tested and
# measured slower on the C4 step (graph replay p50 1.39 -> 1.8-2.2 ms with
# write-through slabs; per call 6.6-13 us vs 5.6-9 us one workgroup per
# tile, tools/decode_ab.py shapes splitk): off.
ROWS_SPLITK = False


def rows_kgroups(N, K, ln):
    """Workgroups per 32-column tile: fill ~256 workgroups, each keeping
    >= 128 of K (one wave trip) and K / kgroups a LayerNorm-prologue size."""
    tiles = -(-N // 32)
    if not ROWS_SPLITK or tiles > ROWS_MAX_TILES:
        return 1
    kg = 1
    while tiles * kg < 256 and kg < ROWS_MAX_KG and K % (64 * kg * 2) == 0 and K // (kg * 2) >= 128:
        kg *= 2
    if ln:
        while kg > 1 and not gemm_rows_ln_ok(K // kg):
            kg //= 2
    return kg


def gemm_rows(x, weight, bias=None, act=None, conv=None, ln=None, res=None, packed_out=None, u_packed=False):
    """y = act(x @ weight.t() + bias) for the decode step's skinny GEMMs
    (x: M <= 32 rows, bf16; act None or "gelu" = exact-erf F.gelu).

    conv = (conv_state (M, C, 4) fp32, conv_w (C, 4) fp32, conv_b or None):
        columns [0, C) also pass through causal_conv1d_update + SiLU;
        returns (y, u) with u (M, C) bf16.
    ln = (w, b, eps[, gamma, beta]): the x operand is LayerNorm'd (+FiLM) on
        the fly, exactly as ops.layer_norm would produce it.
    res: (M, N) bf16; y = bf16(y + res) (the residual stream after the add).
    x may be a PackedAct (with a PackedRows weight): coalesced operand loads.
    packed_out "only" / "also": y comes back as a PackedAct (instead of /
        besides the row-major tensor: (y, y_packed)) for the next projection.
    u_packed: with conv, also a PackedAct of u (returned last).
    """
    packed = isinstance(weight, PackedRows)
    xpk = isinstance(x, PackedAct)
    _check_cuda(x.data if xpk else x, weight.data if packed else weight, bias)
    if not gemm_rows_ok(x, weight):
        raise ValueError(f"gemm_rows: unsupported operands x{tuple(x.shape)}/{'packed' if xpk else x.stride()} "
                         f"w{tuple(weight.shape)}/{'packed' if packed else weight.stride()}")
    M, K = x.shape
    N = weight.shape[0]
    if weight.shape[1] != K:
        raise ValueError("gemm_rows: K mismatch")
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
        if bias.numel() != N:
            raise ValueError("gemm_rows: bias size")
    dev = x.data.device if xpk else x.device
    y = None if packed_out == "only" else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    yp = PackedAct.empty(M, N, dev) if packed_out else None
    a = L.RowsArgs()
    a.M, a.N, a.K, a.act = M, N, K, {None: 0, "gelu": 1}[act]
    a.ldx, a.ldw, a.ldy = 0 if xpk else x.stride(0), 0 if packed else weight.stride(0), N if y is None else y.stride(0)
    a.x, a.W, a.bias, a.y = (x.data if xpk else x).data_ptr(), (weight.data if packed else weight).data_ptr(), \
        L.ptr(bias), L.ptr(y)
    a.w_packed, a.x_packed = int(packed), int(xpk)
    if yp is not None:
        a.y_packed = yp.data.data_ptr()
    out = [yp] if y is None else ([y, yp] if yp is not None else [y])
    if conv is not None:
        cs, cw, cb = conv
        C = cw.shape[0]
        if cs.dtype != torch.float32 or cs.shape != (M, C, 4) or not cs.is_contiguous() or cw.shape != (C, 4):
            raise ValueError("gemm_rows: conv state must be (M, C, 4) fp32 contiguous, weight (C, 4)")
        u = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        a.conv_dim, a.conv_state, a.conv_w, a.conv_b = C, cs.data_ptr(), cw.data_ptr(), L.ptr(cb)
        a.u, a.ldu = u.data_ptr(), u.stride(0)
        out.append(u)
        if u_packed:
            up = PackedAct.empty(M, C, dev)
            a.u_packed = up.data.data_ptr()
            out.append(up)
    if ln is not None:
        lw, lb, eps = ln[0], ln[1], ln[2]
        if lw.dtype != torch.float32 or lb.dtype != torch.float32 or lw.numel() != K or not lw.is_contiguous():
            raise ValueError("gemm_rows: LayerNorm weight / bias must be contiguous fp32 of length K")
        a.ln_w, a.ln_b, a.ln_eps = lw.data_ptr(), lb.data_ptr(), float(eps)
        if len(ln) > 3 and ln[3] is not None:
            g, be = ln[3], ln[4]
            if xpk:   # packed x: FiLM rows as packed images too
                if not (isinstance(g, PackedAct) and isinstance(be, PackedAct) and g.shape == be.shape == (M, K)):
                    raise ValueError("gemm_rows: with a packed x, FiLM gamma / beta must be PackedAct (M, K)")
                a.gamma, a.beta, a.ld_gb = g.data.data_ptr(), be.data.data_ptr(), 0
            else:
                if g.dtype != torch.bfloat16 or g.stride() != be.stride() or g.shape != (M, K):
                    raise ValueError("gemm_rows: FiLM gamma / beta must be (M, K) bf16 with equal strides")
                a.gamma, a.beta, a.ld_gb = g.data_ptr(), be.data_ptr(), g.stride(0)
    if res is not None:
        if res.dtype != torch.bfloat16 or res.shape != (M, N) or res.stride(1) != 1:
            raise ValueError("gemm_rows: res must be (M, N) bf16 with unit column stride")
        a.res, a.ld_res = res.data_ptr(), res.stride(0)
    kg = 1 if packed else rows_kgroups(N, K, ln is not None)
    if kg > 1:
        slab, cnt = rows_workspace(dev)
        a.kgroups, a.splitk_slab, a.splitk_count = kg, slab.data_ptr(), cnt.data_ptr()
    L.call("mtts_gemm_rows", a)
    return out[0] if len(out) == 1 else tuple(out)
