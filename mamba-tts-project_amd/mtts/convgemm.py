"""Direct fp32 convolutions and projections of the text encoder / duration
predictor on the windowed-row MFMA GEMM (csrc/convgemm.hip, mtts_convgemm).

Reference sites: FastSpeech2's PositionwiseFeedForward (Conv1d k = 9 -> ReLU
-> Conv1d k = 1), VariancePredictor (Conv k = 3, padding 1, twice), the
MultiHeadAttention projections (w_qs / w_ks / w_vs / fc) and the
VariancePredictor's linear layer -- reached from /root/reference/
text_encoder.py:80-85 (FFT blocks), 118-122 (encoder) and 131-209 (duration
predictor).  All fp32 as the reference runs them.

A convolution over channel-last x (B, T, C) with weight (O, C, K), padding p
(2p = K - 1, the reference's 'same' convolutions):
  forward   y[b, t] = W(O, K*C) . x_pad[b, t .. t+K-1, :]          NT, windowed A
  data grad dx[b, s] = Wflip(C, K*O) . dy_pad[b, s .. s+K-1, :]    NT, windowed A
  weight    dW(O, K*C) = dy^T . window(x_pad)                       TN, windowed B
No unfold copy: the zero-padded activation's rows overlap as GEMM rows.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn.functional as F

from . import _lib as L
from .linear import colsum

NT, TN = 0, 1
EPI_BIAS, EPI_RELU, EPI_DRELU = 1, 2, 4


def _map(t: torch.Tensor, seg_rows: int, seg_stride: int, row_stride: int) -> L.RowMap:
    return L.RowMap(t.data_ptr(), seg_rows, seg_stride, row_stride)


def _plain(t2: torch.Tensor) -> L.RowMap:
    """A (rows, cols) matrix with unit column stride."""
    assert t2.stride(-1) == 1
    return _map(t2, t2.shape[0], 0, t2.stride(0))


def _window(xp: torch.Tensor, T: int) -> L.RowMap:
    """Rows b*T + t of the windows xp[b, t .. t+K-1, :] of a contiguous (B, T + K - 1, C) tensor."""
    _, Tp, C = xp.shape
    return _map(xp, T, Tp * C, C)


TILE, BK = 128, 32


def splits_for(m, n, k):
    """K split: ~512 workgroups (two per CU) when the output has fewer
    128 x 128 tiles, each split keeping >= 8 K-steps of 32."""
    tiles = -(-m // TILE) * -(-n // TILE)
    return max(1, min(512 // tiles, (-(-k // BK)) // 8, 16))


def gemm(layout, m, n, k, a, b, c, bias=None, epilogue=0, aux=None, beta=0.0, device="cuda"):
    """One mtts_convgemm call on the current stream (the tensors the maps
    point into are kept alive by the caller until it returns)."""
    args = L.ConvGemmArgs()
    args.layout, args.m, args.n, args.k = layout, m, n, k
    args.a, args.b, args.c = a, b, c
    if aux is not None:
        args.aux = aux
    args.bias = 0 if bias is None else bias.data_ptr()
    args.epilogue, args.beta = epilogue, beta
    args.splits = splits_for(m, n, k)
    ws = None
    if args.splits > 1:
        ws = torch.empty(L.lib().mtts_convgemm_workspace(C.byref(args)), device=device, dtype=torch.uint8)
        args.workspace = ws.data_ptr()
    L.call("mtts_convgemm", args)


def _f32c(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"convgemm: fp32 only (got {t.dtype})")
    return t.contiguous()


def _pad(x: torch.Tensor, p: int) -> torch.Tensor:
    return F.pad(x, (0, 0, p, p)) if p else x


def conv_forward(x, weight, bias, relu):
    """y (B, T, O) = [relu](conv(x, weight) + bias); x (B, T, C) contiguous fp32."""
    B, T, C = x.shape
    O, _, K = weight.shape
    p = (K - 1) // 2
    xp = _pad(x, p)
    wf = weight.permute(0, 2, 1).reshape(O, K * C) if K > 1 else weight.view(O, C)
    wf = wf.contiguous()
    y = torch.empty(B, T, O, device=x.device, dtype=torch.float32)
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_RELU if relu else 0)
    gemm(NT, B * T, O, K * C, _window(xp, T), _plain(wf), _plain(y.view(B * T, O)), bias=bias, epilogue=epi)
    return y, xp


def conv_backward(dy, xp, weight, need_dx, need_dw, need_db, relu_out=None):
    """Gradients of y = conv(x) (+ bias) for dy (B, T, O); with `relu_out` (the
    forward's ReLU output) dy is first masked by relu_out > 0 -- that mask is
    fused into the data-gradient epilogue of the layer that PRODUCED dy when
    the caller does it (ConvFFNFn), else applied here."""
    B, T, O = dy.shape
    _, C, K = weight.shape
    p = (K - 1) // 2
    if relu_out is not None:
        dy = torch.where(relu_out > 0, dy, torch.zeros((), device=dy.device))
    dy = dy.contiguous()
    dx = dw = db = None
    if need_dx:
        wd = weight.flip(2).permute(1, 2, 0).reshape(C, K * O).contiguous() if K > 1 else \
            weight.view(O, C).t().contiguous()
        dyp = _pad(dy, p)
        dx = torch.empty(B, T, C, device=dy.device, dtype=torch.float32)
        gemm(NT, B * T, C, K * O, _window(dyp, T), _plain(wd), _plain(dx.view(B * T, C)))
    if need_dw:
        dwf = torch.empty(O, K * C, device=dy.device, dtype=torch.float32)
        gemm(TN, O, K * C, B * T, _plain(dy.view(B * T, O)), _window(xp, T), _plain(dwf))
        dw = dwf.view(O, K, C).permute(0, 2, 1).contiguous() if K > 1 else dwf.view(O, C, 1)
    if need_db:
        db = colsum(dy.view(B * T, O))
    return dx, dw, db


class Conv1dFn(torch.autograd.Function):
    """y = [relu](conv1d_same(x, weight) + bias), channel-last fp32."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        y, xp = conv_forward(x, weight, bias, relu)
        ctx.relu = relu
        ctx.save_for_backward(xp, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, weight, y = ctx.saved_tensors
        need = ctx.needs_input_grad
        dx, dw, db = conv_backward(dy, xp, weight, need[0], need[1], need[2], relu_out=y if ctx.relu else None)
        return dx, dw, db, None


class ConvFFNFn(torch.autograd.Function):
    """FastSpeech2 PositionwiseFeedForward's convolutions:
    out = conv2(relu(conv1(x) + b1)) + b2, the ReLU backward fused into
    conv2's data-gradient epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        h, xp = conv_forward(x, w1, b1, True)
        out, hp = conv_forward(h, w2, b2, False)
        ctx.save_for_backward(xp, w1, hp, w2)
        ctx.has_b = (b1 is not None, b2 is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        xp, w1, hp, w2 = ctx.saved_tensors
        need = ctx.needs_input_grad
        dout = dout.contiguous()
        B, T, O = dout.shape
        _, H, K2 = w2.shape
        p2 = (K2 - 1) // 2
        h = hp[:, p2:p2 + T] if p2 else hp
        # dh = (dout conv2^T) * (h > 0): conv2's data gradient with the ReLU mask in its epilogue
        wd2 = w2.flip(2).permute(1, 2, 0).reshape(H, K2 * O).contiguous() if K2 > 1 else \
            w2.view(O, H).t().contiguous()
        dyp = _pad(dout, p2)
        dh = torch.empty(B, T, H, device=dout.device, dtype=torch.float32)
        hc = h.contiguous()
        gemm(NT, B * T, H, K2 * O, _window(dyp, T), _plain(wd2), _plain(dh.view(B * T, H)),
             epilogue=EPI_DRELU, aux=_plain(hc.view(B * T, H)))
        _, dw2, db2 = conv_backward(dout, hp, w2, False, need[3], need[4] and ctx.has_b[1])
        dx, dw1, db1 = conv_backward(dh, xp, w1, need[0], need[1], need[2] and ctx.has_b[0])
        return dx, dw1, db1, dw2, db2


def conv1d_same(x, weight, bias=None, relu=False):
    """'same' Conv1d (2 * padding = K - 1) on channel-last fp32 x (B, T, C)."""
    x = _f32c(x)
    return Conv1dFn.apply(x, weight, bias, relu)


def conv_ffn(x, w1, b1, w2, b2):
    return ConvFFNFn.apply(_f32c(x), w1, b1, w2, b2)


class LinearFn(torch.autograd.Function):
    """fp32 y = x W^T + b over the last axis (a k = 1 convolution)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        O = weight.shape[0]
        y = torch.empty(x2.shape[0], O, device=x.device, dtype=torch.float32)
        gemm(NT, x2.shape[0], O, shp[-1], _plain(x2), _plain(weight), _plain(y), bias=bias,
             epilogue=EPI_BIAS if bias is not None else 0)
        ctx.save_for_backward(x2, weight)
        ctx.has_b = bias is not None
        return y.view(*shp[:-1], O)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        O, C = weight.shape
        dy2 = dy.reshape(-1, O).contiguous()
        need = ctx.needs_input_grad
        dx = dw = db = None
        if need[0]:
            wt = weight.t().contiguous()
            dx = torch.empty(x2.shape[0], C, device=dy.device, dtype=torch.float32)
            gemm(NT, x2.shape[0], C, O, _plain(dy2), _plain(wt), _plain(dx))
            dx = dx.view(*dy.shape[:-1], C)
        if need[1]:
            dw = torch.empty(O, C, device=dy.device, dtype=torch.float32)
            gemm(TN, O, C, x2.shape[0], _plain(dy2), _plain(x2), _plain(dw))
        if need[2] and ctx.has_b:
            db = colsum(dy2)
        return dx, dw, db


def linear(x, weight, bias=None):
    """fp32 x W^T + b; an output width not a multiple of 4 (the duration
    predictor's 1-wide head) runs on zero-padded weight rows."""
    x = _f32c(x)
    O = weight.shape[0]
    if O % 4:
        pad = 4 - O % 4
        w4 = F.pad(weight, (0, 0, 0, pad))
        b4 = F.pad(bias, (0, pad)) if bias is not None else None
        return LinearFn.apply(x, w4, b4)[..., :O]
    return LinearFn.apply(x, weight.contiguous(), bias)
