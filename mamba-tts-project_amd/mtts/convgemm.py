"""Direct fp32 convolutions and projections of the text encoder / duration
predictor on the windowed-row MFMA GEMM (csrc/convgemm.hip, mtts_convgemm).

Reference sites: FastSpeech2's PositionwiseFeedForward (Conv1d k = 9 -> ReLU
-> Conv1d k = 1), VariancePredictor (Conv k = 3, padding 1, twice), the
MultiHeadAttention projections (w_qs / w_ks / w_vs / fc) and the
VariancePredictor's linear layer -- reached from /root/reference/
text_encoder.py:80-85 (FFT blocks), 118-122 (encoder) and 131-209 (duration
predictor).  All fp32 as the reference runs them.

A convolution over channel-last x (B, T, C) with weight (O, C, K), padding p
(2p = K - 1, the reference's 'same' convolutions) and Wf = W as (O, K*C)
([o][k][c], made once by the forward and kept for the backward):
  forward   y[b, t] = Wf . x_pad[b, t .. t+K-1, :]                 NT, windowed A
  data grad dx[b, s] = sum_{j,o} dy_pad[b, s + j, o] Wf[o][K-1-j]   NN, windowed A,
            B row (j, o) = Wf[o, (K-1-j) C ..] (a row map with a negative segment stride)
  weight    dWf = dy^T . window(x_pad)                              TN, windowed B
No unfold copy (the zero-padded activation's rows overlap as GEMM rows) and
no transposed / flipped weight copy.  With C % 32 == 0 (every text-encoder
convolution) there is no padded copy either: x_pad is virtual, a halo row map
over x whose out-of-sequence taps the kernel reads as zeros.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn.functional as F

from . import _lib as L
from .linear import colsum

NT, TN, NN = 0, 1, 2
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


def _halo_window(x: torch.Tensor, p: int) -> L.RowMap:
    """The same windows over the UNPADDED (B, T, C) x: a halo map (mtts.h
    MttsRowMap), taps outside [0, T) read 0 in the kernel -- no padded copy."""
    _, T, C = x.shape
    m = _map(x, T, T * C, C)
    m.halo_c, m.halo_p = C, p
    return m


def _halo_ok(C, p):
    return p > 0 and C % 32 == 0


def _win(x: torch.Tensor, T: int, K: int) -> L.RowMap:
    """Conv windows of x: padded (B, T + K - 1, C) or unpadded (halo)."""
    return _window(x, T) if x.shape[1] != T or K == 1 else _halo_window(x, (K - 1) // 2)


def _pad_for(x: torch.Tensor, p: int) -> torch.Tensor:
    """x itself where the kernel zero-pads (halo), else a padded copy."""
    return x if (p == 0 or _halo_ok(x.shape[2], p)) else F.pad(x, (0, 0, p, p))


TILE, BK = 128, 32


FORCE_SPLITS = None    # measurement hook (tools/convgemm_bench.py SPLITS=...)
WG_TARGET = 1024       # workgroups to aim for: 2 resident per CU, 2 rounds


def splits_for(m, n, k):
    """K split: one workgroup per 128 x 128 tile is latency-bound (one
    workgroup per CU overlaps nothing: the k = 9 conv forward runs 370 us
    unsplit, 133 us in 8 splits, tools/convgemm_bench.py SPLITS sweep,
    profiles/r05_convgemm_splits.txt), so aim for ~1024 workgroups (two
    resident per CU and fine-grained enough to balance), up to 16 splits of
    >= 4 K-steps each.  The slab sum moves 8 bytes per output element per
    split, so wide outputs stop at max(4, 8M / (m n)) splits (k = 9 forward,
    1M outputs: 8 splits 133 us vs 16 splits 144 us)."""
    tiles = -(-m // TILE) * -(-n // TILE)
    nk = -(-k // BK)
    return max(1, min(16, -(-WG_TARGET // tiles), nk // 4, max(4, (8 << 20) // (m * n))))


def gemm(layout, m, n, k, a, b, c, bias=None, epilogue=0, aux=None, beta=0.0, device="cuda", colsum_a=None):
    """One mtts_convgemm call on the current stream (the tensors the maps
    point into are kept alive by the caller until it returns).  colsum_a (TN,
    fp32 (m,)): receives the column sums of A over the k rows."""
    args = L.ConvGemmArgs()
    args.layout, args.m, args.n, args.k = layout, m, n, k
    args.a, args.b, args.c = a, b, c
    if aux is not None:
        args.aux = aux
    args.bias = 0 if bias is None else bias.data_ptr()
    args.epilogue, args.beta = epilogue, beta
    args.splits = splits_for(m, n, k) if FORCE_SPLITS is None else FORCE_SPLITS
    if colsum_a is not None:
        args.colsum_a = colsum_a.data_ptr()
    ws = None
    if args.splits > 1:
        ws = torch.empty(L.lib().mtts_convgemm_workspace(C.byref(args)), device=device, dtype=torch.uint8)
        args.workspace = ws.data_ptr()
    L.call("mtts_convgemm", args)


def _f32c(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"convgemm: fp32 only (got {t.dtype})")
    return t.contiguous()


def _wf(weight):
    O, C, K = weight.shape
    return weight.view(O, C) if K == 1 else weight.permute(0, 2, 1).reshape(O, K * C).contiguous()


def conv_forward(x, weight, bias, relu):
    """y (B, T, O) = [relu](conv(x, weight) + bias); x (B, T, C) contiguous fp32.
    Returns (y, x_pad, Wf)."""
    B, T, C = x.shape
    O, _, K = weight.shape
    p = (K - 1) // 2
    xp = _pad_for(x, p)
    wf = _wf(weight)
    y = torch.empty(B, T, O, device=x.device, dtype=torch.float32)
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_RELU if relu else 0)
    gemm(NT, B * T, O, K * C, _win(xp, T, K), _plain(wf), _plain(y.view(B * T, O)), bias=bias, epilogue=epi)
    return y, xp, wf


def _wflip_map(wf, K):
    """B rows (j, o) = Wf[o, (K-1-j) C : (K-j) C] of the data gradient."""
    O, KC = wf.shape
    C = KC // K
    base = wf[:, (K - 1) * C:] if K > 1 else wf
    return _map(base, O, -C, KC)


def dgrad(dy, wf, K, epilogue=0, aux=None):
    """dx (B, T, C) of a 'same' convolution for dy (B, T, O) contiguous."""
    B, T, O = dy.shape
    C = wf.shape[1] // K
    dyp = _pad_for(dy, (K - 1) // 2)
    dx = torch.empty(B, T, C, device=dy.device, dtype=torch.float32)
    gemm(NN, B * T, C, K * O, _win(dyp, T, K), _wflip_map(wf, K), _plain(dx.view(B * T, C)), epilogue=epilogue,
         aux=aux)
    return dx


def conv_backward(dy, xp, wf, K, need_dx, need_dw, need_db, relu_out=None):
    """Gradients of y = conv(x) (+ bias) for dy (B, T, O); with `relu_out` (the
    forward's ReLU output) dy is first masked by relu_out > 0 (ConvFFNFn fuses
    that mask into the data-gradient epilogue of the layer that produced dy
    instead).  Returns dx, dW (O, C, K), db."""
    B, T, O = dy.shape
    C = wf.shape[1] // K
    if relu_out is not None:
        dy = torch.where(relu_out > 0, dy, torch.zeros((), device=dy.device))
    dy = dy.contiguous()
    dx = dw = db = None
    if need_dx:
        dx = dgrad(dy, wf, K)
    if need_dw:
        dwf = torch.empty(O, K * C, device=dy.device, dtype=torch.float32)
        if need_db:   # the bias gradient from the weight-gradient kernel's own dy tiles
            db = torch.empty(O, device=dy.device, dtype=torch.float32)
        gemm(TN, O, K * C, B * T, _plain(dy.view(B * T, O)), _win(xp, T, K), _plain(dwf), colsum_a=db)
        # (O, C, K) over the [o][k][c] result, no transposing copy: a weight
        # kept [O][K][C] (text_encoder.kc_major) takes it as its gradient as is;
        # autograd re-lays it out for a contiguous weight
        dw = dwf.view(O, K, C).permute(0, 2, 1) if K > 1 else dwf.view(O, C, 1)
    if need_db and db is None:
        db = colsum(dy.view(B * T, O))
    return dx, dw, db


class Conv1dFn(torch.autograd.Function):
    """y = [relu](conv1d_same(x, weight) + bias), channel-last fp32."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        y, xp, wf = conv_forward(x, weight, bias, relu)
        ctx.relu, ctx.K = relu, weight.shape[2]
        ctx.save_for_backward(xp, wf, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, wf, y = ctx.saved_tensors
        need = ctx.needs_input_grad
        dx, dw, db = conv_backward(dy, xp, wf, ctx.K, need[0], need[1], need[2], relu_out=y if ctx.relu else None)
        return dx, dw, db, None


class ConvFFNFn(torch.autograd.Function):
    """FastSpeech2 PositionwiseFeedForward's convolutions:
    out = conv2(relu(conv1(x) + b1)) + b2, the ReLU backward fused into
    conv2's data-gradient epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        h, xp, wf1 = conv_forward(x, w1, b1, True)
        out, hp, wf2 = conv_forward(h, w2, b2, False)
        ctx.save_for_backward(xp, wf1, hp, wf2)
        ctx.K = (w1.shape[2], w2.shape[2])
        ctx.has_b = (b1 is not None, b2 is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        xp, wf1, hp, wf2 = ctx.saved_tensors
        K1, K2 = ctx.K
        need = ctx.needs_input_grad
        dout = dout.contiguous()
        B, T, O = dout.shape
        p2 = (K2 - 1) // 2
        h = (hp[:, p2:p2 + T] if hp.shape[1] != T else hp).contiguous()
        # dh = (dout conv2^T) * (h > 0): conv2's data gradient with the ReLU mask in its epilogue
        dh = dgrad(dout, wf2, K2, epilogue=EPI_DRELU, aux=_plain(h.view(B * T, h.shape[2])))
        _, dw2, db2 = conv_backward(dout, hp, wf2, K2, False, need[3], need[4] and ctx.has_b[1])
        dx, dw1, db1 = conv_backward(dh, xp, wf1, K1, need[0], need[1], need[2] and ctx.has_b[0])
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
        if need[0]:   # NN: the weight's rows are the k-rows, no transpose copy
            dx = torch.empty(x2.shape[0], C, device=dy.device, dtype=torch.float32)
            gemm(NN, x2.shape[0], C, O, _plain(dy2), _plain(weight), _plain(dx))
            dx = dx.view(*dy.shape[:-1], C)
        if need[1]:
            dw = torch.empty(O, C, device=dy.device, dtype=torch.float32)
            if need[2] and ctx.has_b:   # from the weight-gradient kernel's own dy tiles
                db = torch.empty(O, device=dy.device, dtype=torch.float32)
            gemm(TN, O, C, x2.shape[0], _plain(dy2), _plain(x2), _plain(dw), colsum_a=db)
        if need[2] and ctx.has_b and db is None:
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
