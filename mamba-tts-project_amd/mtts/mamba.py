"""Mamba v1 mixer on libmtts (the build's replacement for `mamba_ssm.Mamba`).

Reference contract: mamba_decoder.py:10-15 documents
    out, new_state = mamba(x)          # full sequence, state from h = 0
    out, new_state = mamba(x, state)   # incremental (decode) step
with x (B, T, d_model) and an opaque per-layer state; the build's state is
(conv_state (B, d_inner, d_conv) fp32, ssm_state (B, d_inner, d_state) fp32),
the [upstream] mamba-ssm InferenceParams layout.  Parameters, names, shapes
and initialisation follow [upstream] mamba_ssm/modules/mamba_simple.py
(d_state=16, d_conv=4, expand=2, dt_rank=ceil(d/16), bias=False,
conv_bias=True, dt in [1e-3, 1e-1], A_log = log(1..16), D = 1), so a
reference state_dict loads unchanged.

Hot path (all HIP through the C ABI, GEMMs through torch):
  xz = in_proj(x)                         (B, L, 2*di)   channel-last
  u  = silu(conv1d(xz[..., :di]))         HIP causal_conv1d (strided view)
  x_dbl = x_proj(u) -> dt | B | C
  delta = dt_proj.weight @ dt             (bias folded into the scan)
  y  = selective_scan(u, delta, A, B, C, D, z = xz[..., di:])   HIP
  out = out_proj(y)
Backward (MambaInnerFn) runs the HIP scan/conv backward kernels and writes
dz and dx straight into one d(xz) buffer (no concat).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import gemm as G
from . import ops
from . import wgrad as WG
from .linear import cast_scope, cast_weight, cast_weight_t, linear, wgrad


class MambaInnerFn(torch.autograd.Function):
    """(xz, params[, state]) -> (y, conv_state, ssm_state); y is pre-out_proj."""

    @staticmethod
    def forward(ctx, xz, conv_w, conv_b, W_x, W_dt, A_log, D, dt_bias, conv_state_in, h0):
        cd = xz.dtype
        di = xz.shape[-1] // 2
        N = A_log.shape[1]
        r = W_dt.shape[1]
        Wx, Wdt = cast_weight(W_x, cd), cast_weight(W_dt, cd)
        x, z = xz[..., :di], xz[..., di:]
        u, conv_state = ops.conv_fwd(x, conv_w, conv_b, True, state_in=conv_state_in, want_state=True)
        u2 = u.view(-1, di)
        # x_proj stays on hipBLASLt (21 us vs 25 for SKINNY_N at C2, tools/skinny_ab.py);
        # dt_proj on the SMALL_K MFMA kernel (csrc/skinny.hip) when the shapes allow
        x_dbl = (G.mm_skinny(u2, Wx) if G.SKINNY_XPROJ and G.skinny_ok(u2, Wx) else u2 @ Wx.t()).view(
            *u.shape[:-1], r + 2 * N)
        dt, Bm, Cm = x_dbl[..., :r], x_dbl[..., r:r + N], x_dbl[..., r + N:]
        dt2 = x_dbl.view(-1, r + 2 * N)[:, :r]
        delta = (G.mm_skinny(dt2, Wdt) if G.SKINNY_DTPROJ and G.skinny_ok(dt2, Wdt) else dt2 @ Wdt.t()).view(
            *u.shape[:-1], di)
        # A = -exp(A_log) is formed inside the scan kernels (a_is_log): no per-layer exp / neg launches
        A_log32 = A_log.detach().float().contiguous()
        need = any(ctx.needs_input_grad)
        y, last, ckpt = ops.scan_fwd(u, delta, A_log32, Bm, Cm, D, z, dt_bias, True, h0, want_last=True,
                                     want_ckpt=need, a_is_log=True)
        if need:
            ctx.save_for_backward(xz, conv_w, conv_b, W_x, W_dt, A_log, D, dt_bias, u, x_dbl, delta, ckpt,
                                  conv_state_in, h0, A_log32)
        ctx.mark_non_differentiable(conv_state, last)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the unused state outputs
        return y, conv_state, last

    @staticmethod
    def backward(ctx, dy, _dconv, _dlast):
        (xz, conv_w, conv_b, W_x, W_dt, A_log, D, dt_bias, u, x_dbl, delta, ckpt,
         conv_state_in, h0, A_log32) = ctx.saved_tensors
        if dy is None:   # grads are not materialised: y unused downstream
            dy = torch.zeros(xz.shape[:-1] + (xz.shape[-1] // 2,), device=xz.device, dtype=xz.dtype)
        cd = u.dtype
        Wx, Wdt = cast_weight(W_x, cd), cast_weight(W_dt, cd)
        di = xz.shape[-1] // 2
        N = A_log.shape[1]
        r = W_dt.shape[1]
        Bsz, Ln, _ = xz.shape
        x, z = xz[..., :di], xz[..., di:]
        dt, Bm, Cm = x_dbl[..., :r], x_dbl[..., r:r + N], x_dbl[..., r + N:]
        dxz = torch.empty_like(xz)
        dx_dbl = torch.empty(Bsz, Ln, r + 2 * N, device=xz.device, dtype=torch.float32)
        need_dh0 = h0 is not None and ctx.needs_input_grad[9]
        du, ddelta, _, _, _, dA_log, dD, dbias, dh0 = ops.scan_bwd(
            u, delta, A_log32, Bm, Cm, D, z, dt_bias, True, h0, ckpt, dy,
            dz=dxz[..., di:], dB=dx_dbl[..., r:r + N], dC=dx_dbl[..., r + N:], need_dh0=need_dh0, a_is_log=True)
        # dt_proj: delta = dt @ W_dt^T  ->  d(dt) = d(delta) W_dt (fp32, into d(x_dbl)), dW_dt
        dd2 = ddelta.reshape(-1, di)
        dxd2 = dx_dbl.view(-1, r + 2 * N)
        WdtT = cast_weight_t(W_dt, cd) if cd == torch.bfloat16 else None   # (r, di): k-contiguous
        if WdtT is not None and G.skinny_ok(dd2, WdtT, out_dtype=torch.float32, out=dxd2[:, :r]):
            G.mm_skinny(dd2, WdtT, out=dxd2[:, :r])
        else:
            dx_dbl[..., :r] = (ddelta @ Wdt).float()
        dt2 = x_dbl.view(-1, r + 2 * N)[:, :r]
        # the skinny weight gradients ride in the layer's grouped launch when
        # deferral is on (mtts.wgrad: 16 tiles in otherwise idle CUs)
        dW_dt = None
        if not WG.submit([(dd2, dt2, W_dt, None)], narrow=True):
            dW_dt = G.mm_skinny_tn(dd2, dt2) if G.skinny_tn_ok(dd2, dt2) else wgrad(dd2, dt2)
        # x_proj: x_dbl = u @ W_x^T  ->  du += d(x_dbl) W_x (accumulated by the GEMM), dW_x
        gx = dx_dbl.to(cd).view(-1, r + 2 * N)
        du2 = du.view(-1, di)
        WxT = cast_weight_t(W_x, cd) if cd == torch.bfloat16 else None     # (di, r + 2N): k-contiguous
        if WxT is not None and G.SKINNY_DU and G.skinny_ok(gx, WxT, out=du2):
            G.mm_skinny(gx, WxT, out=du2, beta=1.0)
        else:
            du2.addmm_(gx, Wx)
        u2 = u.reshape(-1, di)
        dW_x = None
        if not WG.submit([(gx, u2, W_x, None)], narrow=True):
            dW_x = G.mm_skinny_tn(u2, gx, trans_c=True) if G.skinny_tn_ok(u2, gx) else wgrad(gx, u2)
        # the conv's left history (a prefilled conv_state) enters the
        # recomputed pre-activations and the weight gradient
        _, dw, db = ops.conv_bwd(x, conv_w, conv_b, du, True, dx=dxz[..., :di], state_in=conv_state_in)
        dstate = None
        if conv_state_in is not None and ctx.needs_input_grad[8]:
            dstate = _conv_state_grad(x, conv_w, conv_b, conv_state_in, du)
        dA_log = dA_log.to(A_log.dtype)
        return (dxz, dw.reshape(conv_w.shape).to(conv_w.dtype), db.to(conv_b.dtype),
                None if dW_x is None else dW_x.to(W_x.dtype), None if dW_dt is None else dW_dt.to(W_dt.dtype),
                dA_log, dD.to(D.dtype), dbias.to(dt_bias.dtype), dstate,
                None if dh0 is None else dh0.to(h0.dtype))


def _conv_state_grad(x, conv_w, conv_b, state, du):
    """d conv_state (B, D, K): the history column j (time j - K) feeds the
    pre-activations of the first K - 1 steps with weight w[j - 1 - t]
    (out[t] = sum_k w[k] [state | x][t + 1 + k]).  O(B * D * K^2) on the
    first K - 1 steps only, so a few tiny device ops."""
    K = state.shape[-1]
    di = state.shape[1]
    w = conv_w.reshape(di, K).float()
    L = x.shape[1]
    n = min(K - 1, L)
    full = torch.cat([state.float(), x[:, :n].transpose(1, 2).float()], dim=-1)   # (B, D, K + n)
    pre = torch.stack([(full[:, :, 1 + t:1 + t + K] * w).sum(-1) for t in range(n)], dim=-1)
    if conv_b is not None:
        pre = pre + conv_b.float()[None, :, None]
    s = torch.sigmoid(pre)
    g = du[:, :n].transpose(1, 2).float() * s * (1 + pre * (1 - s))               # dL/dpre, (B, D, n)
    ds = torch.zeros_like(state, dtype=torch.float32)
    for j in range(1, K):
        for t in range(min(j, n)):
            ds[:, :, j] += w[:, j - 1 - t] * g[:, :, t]
    return ds.to(state.dtype)


class Mamba(nn.Module):
    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001, dt_max=0.1,
                 dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True, bias=False,
                 device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.expand = expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        di = self.d_inner
        self.in_proj = nn.Linear(d_model, di * 2, bias=bias, **fk)
        self.conv1d = nn.Conv1d(di, di, kernel_size=d_conv, groups=di, padding=d_conv - 1, bias=conv_bias, **fk)
        self.x_proj = nn.Linear(di, self.dt_rank + d_state * 2, bias=False, **fk)
        self.dt_proj = nn.Linear(self.dt_rank, di, bias=True, **fk)
        # the per-step weight cast also writes W^T for these two (their data
        # gradients run as d(.) . (W^T)^T on the skinny kernels)
        self.x_proj.weight._mtts_want_t = True
        self.dt_proj.weight._mtts_want_t = True
        dt_init_std = self.dt_rank ** -0.5 * dt_scale
        with torch.no_grad():
            if dt_init == "constant":
                self.dt_proj.weight.fill_(dt_init_std)
            else:
                self.dt_proj.weight.uniform_(-dt_init_std, dt_init_std)
            dt = torch.exp(torch.rand(di, **fk) * (math.log(dt_max) - math.log(dt_min)) + math.log(dt_min))
            dt = dt.clamp(min=dt_init_floor)
            self.dt_proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))
        self.dt_proj.bias._no_reinit = True
        A = torch.arange(1, d_state + 1, dtype=torch.float32, device=device).repeat(di, 1).contiguous()
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(di, device=device))
        self.D._no_weight_decay = True
        self.out_proj = nn.Linear(di, d_model, bias=bias, **fk)

    def _w(self, lin, cd):
        return cast_weight(lin.weight, cd)

    def forward(self, x, state=None):
        """x (B, L, d) -> (out (B, L, d), (conv_state, ssm_state))."""
        if not x.is_cuda:
            raise RuntimeError("mtts.Mamba runs on the HIP kernels only (no CPU path)")
        with cast_scope():
            return self._forward(x, state)

    def _forward(self, x, state):
        Bsz, Ln, _ = x.shape
        if state is not None and Ln == 1:
            return self.step(x, state)
        xz = linear(x, self.in_proj.weight, self.in_proj.bias)
        conv_state_in = h0 = None
        if state is not None:
            conv_state_in, h0 = state
        y, conv_state, ssm_state = MambaInnerFn.apply(
            xz, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight, self.dt_proj.weight,
            self.A_log, self.D, self.dt_proj.bias, conv_state_in, h0)
        out = linear(y, self.out_proj.weight, self.out_proj.bias)
        return out, (conv_state, ssm_state)

    @torch.no_grad()
    def step(self, x, state):
        """One decode step; updates conv_state / ssm_state IN PLACE ([upstream]
        Mamba.step semantics) and returns them."""
        conv_state, ssm_state = state
        cd = x.dtype
        di, N, r = self.d_inner, self.d_state, self.dt_rank
        xz = F.linear(x[:, 0], self._w(self.in_proj, cd))
        xs, z = xz[:, :di], xz[:, di:]
        u = ops.conv_update(xs, conv_state, self.conv1d.weight.detach().reshape(di, -1).float().contiguous(),
                            None if self.conv1d.bias is None else self.conv1d.bias.detach().float(), True)
        x_dbl = F.linear(u, self._w(self.x_proj, cd))
        dt, Bm, Cm = x_dbl[:, :r], x_dbl[:, r:r + N], x_dbl[:, r + N:]
        delta = F.linear(dt, self._w(self.dt_proj, cd))
        A = -torch.exp(self.A_log.detach().float())
        y = ops.state_update(ssm_state, u, delta, A, Bm.contiguous(), Cm.contiguous(), self.D.detach().float(),
                             z, self.dt_proj.bias.detach().float(), True)
        out = F.linear(y, self._w(self.out_proj, cd))
        return out[:, None], (conv_state, ssm_state)
