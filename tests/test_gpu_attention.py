"""HIP cross-attention (mtts_attention_fwd / _bwd) against a float64 PyTorch
restatement of nn.MultiheadAttention's core (softmax(q k^T/sqrt(hd) + kpm) v,
reference call sites mamba_decoder.py:72-77, style_cross_attention.py:125-131).

Tolerances: fp32 I/O runs exact-f32 MFMA, so 2e-5 relative to the output
scale; bf16 I/O rounds P / dS to bf16 before the P.V / dS.K products
(flash-attention practice), checked at 2e-2 of the output scale."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def ref_attention(q, k, v, H, kpm):
    B, T, d = q.shape
    S = k.shape[1]
    hd = d // H
    qh = q.double().view(B, T, H, hd).transpose(1, 2)
    kh = k.double().reshape(B, S, H, hd).transpose(1, 2)
    vh = v.double().reshape(B, S, H, hd).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(hd)
    if kpm is not None:
        s = s.masked_fill(kpm[:, None, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ vh).transpose(1, 2).reshape(B, T, d), torch.logsumexp(s, -1)


def make(B, T, S, H, hd, dtype, seed=0, mask=True, full_mask_batch=None):
    g = torch.Generator(device="cuda").manual_seed(seed)
    d = H * hd
    q = torch.randn(B, T, d, device="cuda", generator=g).to(dtype)
    kv = torch.randn(B, S, 2 * d, device="cuda", generator=g).to(dtype)
    kpm = None
    if mask:
        kpm = torch.rand(B, S, device="cuda", generator=g) < 0.3
        kpm[:, 0] = False
        if full_mask_batch is not None:
            kpm[full_mask_batch] = True
    return q, kv, kpm


def close(got, ref, tol):
    scale = ref.abs().max().item() + 1e-6
    err = (got.double() - ref).abs().max().item()
    assert err <= tol * scale, f"max err {err:.3e} > {tol} * {scale:.3e}"


CASES = [  # B, T, S, H, hd
    (2, 64, 12, 4, 16),
    (3, 70, 20, 4, 16),
    (2, 33, 64, 2, 32),
    (2, 130, 100, 4, 64),
    (2, 256, 128, 8, 128),
    (1, 40, 130, 2, 128),
    (2, 1, 128, 8, 128),
    (1, 5, 300, 2, 64),
    (2, 17, 1, 2, 32),
    # single query (decode step; attn_decode_kernel): every head dim, ragged / long key sides
    (3, 1, 12, 4, 16),
    (2, 1, 5, 2, 32),
    (1, 1, 300, 2, 64),
    (32, 1, 1000, 8, 128),
    # single-pass decode kernel (attn_decode1_kernel, all keys in registers): U = 4 and 8
    (32, 1, 128, 16, 64),
    (4, 1, 200, 4, 64),
    (2, 1, 60, 2, 128),
    (3, 1, 100, 2, 128),
    (2, 1, 33, 4, 16),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
def test_forward_matches_reference(case, dtype):
    from mtts import attn_kernels as A
    B, T, S, H, hd = case
    q, kv, kpm = make(B, T, S, H, hd, dtype, mask=S > 1)
    d = H * hd
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    ref, ref_lse = ref_attention(q, kv[..., :d], kv[..., d:], H, kpm)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    close(out, ref, tol)
    close(lse, ref_lse, 1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("pattern", ["ramp", "steps", "late_spike"])
@pytest.mark.parametrize("case", [(2, 256, 1100, 4, 64), (1, 128, 700, 2, 128), (2, 256, 128, 4, 64),
                                  (1, 256, 100, 2, 128), (2, 300, 700, 4, 64), (1, 520, 333, 2, 32)])
def test_forward_deferred_max_rescales(case, pattern):
    """The bf16 forward kernels defer the running-max update until a row's
    max grows by more than 2^8 (attn.hip softmax_step).  Scores that grow
    along the key axis -- smoothly, in jumps at 32/64-key tile seams, or as
    one late spike -- force rescales on some rows of a wave and deferrals
    on others; the result must still match the float64 reference."""
    from mtts import attn_kernels as A
    B, T, S, H, hd = case
    q, kv, kpm = make(B, T, S, H, hd, torch.float32, seed=3)
    d = H * hd
    j = torch.arange(S, device="cuda", dtype=torch.float32)
    if pattern == "ramp":
        gain = 0.5 + 6.0 * j / S
    elif pattern == "steps":
        gain = 0.5 + 1.5 * torch.div(j, 32, rounding_mode="floor") % 5
    else:
        gain = torch.full_like(j, 0.7)
        gain[int(S * 0.8):int(S * 0.8) + 3] = 9.0
    kv[..., :d] *= gain[None, :, None]
    q *= (0.4 + (torch.arange(T, device="cuda") % 7).float() * 0.3)[None, :, None]
    q, kv = q.to(torch.bfloat16), kv.to(torch.bfloat16)
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    ref, ref_lse = ref_attention(q, kv[..., :d], kv[..., d:], H, kpm)
    close(out, ref, 2e-2)
    close(lse, ref_lse, 1e-2)


@pytest.mark.parametrize("dtype,T,S,hd", [(torch.float32, 40, 24, 16), (torch.bfloat16, 256, 100, 64),
                                          (torch.bfloat16, 256, 700, 64)])
def test_fully_masked_rows_are_nan_and_others_exact(dtype, T, S, hd):
    from mtts import attn_kernels as A
    B, H = 3, 4
    q, kv, kpm = make(B, T, S, H, hd, dtype, full_mask_batch=1)
    d = H * hd
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    assert torch.isnan(out[1]).all()
    assert torch.isinf(lse[1]).all() and (lse[1] < 0).all()
    ref, _ = ref_attention(q, kv[..., :d], kv[..., d:], H, kpm)
    close(out[[0, 2]], ref[[0, 2]], 2e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("T,S,hd", [(200, 333, 64), (256, 1100, 64), (130, 700, 128), (300, 260, 128)])
def test_rows_past_the_ends_are_not_used(T, S, hd):
    """Buffer-addressed K / V / Q / dO rows (long-key forward, dQ and dK/dV
    kernels): q / kv / dout as row views of larger tensors whose rows past
    T / S hold NaN.  Forward and backward must equal the runs on contiguous
    copies bit for bit and stay finite (no row past the end is read into a
    result, whatever the buffer range check does with the scalar offset)."""
    from mtts import attn_kernels as A
    B, H = 2, 4
    q, kv, kpm = make(B, T, S, H, hd, torch.bfloat16, seed=T + S)
    d = H * hd
    pad = 40

    def big(t, rows):
        bt = torch.full((t.shape[0], rows + pad, t.shape[2]), float("nan"), device="cuda", dtype=t.dtype)
        bt[:, :rows] = t
        return bt[:, :rows]

    qv, kvv = big(q, T), big(kv, S)
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    out2, lse2 = A.attention_fwd(qv, kvv[..., :d], kvv[..., d:], H, kpm, want_lse=True)
    assert torch.isfinite(out2).all() and torch.equal(out, out2) and torch.equal(lse, lse2)
    g = torch.Generator(device="cuda").manual_seed(3)
    do = torch.randn(out.shape, device="cuda", generator=g).to(out.dtype)
    r1 = A.attention_bwd(q, kv[..., :d], kv[..., d:], H, kpm, out, lse, do)
    r2 = A.attention_bwd(qv, kvv[..., :d], kvv[..., d:], H, kpm, out2, lse2, big(do, T))
    for a, b in zip(r1, r2):
        assert torch.isfinite(b).all() and torch.equal(a, b)


@pytest.mark.parametrize("S", [24, 128, 200, 1000])
def test_decode_fully_masked_rows_are_nan(S):
    """q_len = 1 (both decode kernels): a fully masked key side gives NaN rows
    and -inf lse like torch MHA; the other batch rows match the reference."""
    from mtts import attn_kernels as A
    B, T, H, hd = 3, 1, 4, 64
    q, kv, kpm = make(B, T, S, H, hd, torch.float32, full_mask_batch=1)
    d = H * hd
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    assert torch.isnan(out[1]).all()
    assert torch.isinf(lse[1]).all() and (lse[1] < 0).all()
    ref, _ = ref_attention(q, kv[..., :d], kv[..., d:], H, kpm)
    close(out[[0, 2]], ref[[0, 2]], 2e-5)


def test_no_mask_and_separate_k_v_tensors():
    from mtts import attn_kernels as A
    B, T, S, H, hd = 2, 50, 37, 4, 32
    q, kv, _ = make(B, T, S, H, hd, torch.float32, mask=False)
    d = H * hd
    k, v = kv[..., :d].contiguous(), kv[..., d:].contiguous()
    out = A.attention(q, k, v, H)
    ref, _ = ref_attention(q, k, v, H, None)
    close(out, ref, 2e-5)


def _grads(q, kv, H, kpm, fused):
    from mtts import attn_kernels as A
    d = q.shape[-1]
    q = q.detach().requires_grad_(True)
    kv = kv.detach().requires_grad_(True)
    if fused:
        o = A.attention_kv(q, kv, H, kpm)
    else:
        o = A.attention(q, kv[..., :d], kv[..., d:], H, kpm)
    g = torch.Generator(device="cuda").manual_seed(5)
    do = torch.randn(o.shape, device="cuda", generator=g).to(o.dtype)
    o.backward(do)
    return o, q.grad, kv.grad, do


def _ref_grads(q, kv, H, kpm, do):
    d = q.shape[-1]
    q = q.detach().double().requires_grad_(True)
    kv = kv.detach().double().requires_grad_(True)
    o, _ = ref_attention(q, kv[..., :d], kv[..., d:], H, kpm)
    o.backward(do.double())
    return q.grad, kv.grad


@pytest.mark.parametrize("chunks", [None, 1, 3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES[:6] + [(1, 5, 300, 2, 64), (3, 1, 12, 4, 16)])
def test_backward_matches_reference(case, dtype, chunks):
    from mtts import _lib as L
    B, T, S, H, hd = case
    q, kv, kpm = make(B, T, S, H, hd, dtype, seed=3)
    with L.override(attn_chunks=chunks):
        o, dq, dkv, do = _grads(q, kv, H, kpm, fused=True)
    rq, rkv = _ref_grads(q, kv, H, kpm, do)
    tol = 5e-5 if dtype == torch.float32 else 3e-2
    close(dq, rq, tol)
    close(dkv, rkv, tol)


def test_backward_separate_kv_and_determinism():
    B, T, S, H, hd = 2, 96, 50, 4, 64
    q, kv, kpm = make(B, T, S, H, hd, torch.bfloat16, seed=9)
    _, dq1, dkv1, do = _grads(q, kv, H, kpm, fused=False)
    _, dq2, dkv2, _ = _grads(q, kv, H, kpm, fused=True)
    assert torch.equal(dq1, dq2) and torch.equal(dkv1, dkv2)
    rq, rkv = _ref_grads(q, kv, H, kpm, do)
    close(dq1, rq, 3e-2)
    close(dkv1, rkv, 3e-2)


def test_north_star_shape_bf16():
    """C2 decoder shape: B=8, T_audio=2048, T_text=128 (10 % padded), d=1024, H=8."""
    B, T, S, H, hd = 8, 2048, 128, 8, 128
    q, kv, _ = make(B, T, S, H, hd, torch.bfloat16, seed=11, mask=False)
    kpm = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    kpm[:, int(S * 0.9):] = True
    o, dq, dkv, do = _grads(q, kv, H, kpm, fused=True)
    # reference on two batches (float64 on the full batch is slow but fine)
    rq, rkv = _ref_grads(q[:2], kv[:2], H, kpm[:2], do[:2])
    close(dq[:2], rq, 3e-2)
    close(dkv[:2], rkv, 3e-2)


@pytest.mark.parametrize("path", ["split", "split_generic", "fused"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(1, 100, 1100, 2, 128), (2, 64, 777, 4, 64), (2, 33, 129, 2, 32),
                                  (1, 300, 260, 2, 128), (1, 300, 700, 2, 64), (2, 160, 300, 8, 64)])
def test_backward_long_key_side(case, dtype, path):
    """Key side longer than one key group (the train.py shape: 5k reference
    keys): the split backward (dQ launch -- wave-per-query-slice kernel for
    bf16 hd 64/128, or the generic key-split mode-2 kernel -- then the
    per-key-group dK/dV launch: register-resident K / V kernel for bf16 hd 64,
    or the generic mode 1; (1, 300, 700, 2, 64) runs it over query chunks
    into partials) and the fused chunked one all match (paths forced with
    mtts_set_override: attn_bwd, attn_generic)."""
    from mtts import _lib as L
    B, T, S, H, hd = case
    q, kv, kpm = make(B, T, S, H, hd, dtype, seed=5)
    force = {"split": dict(attn_bwd=L.ATTN_BWD_SPLIT), "split_generic": dict(attn_bwd=L.ATTN_BWD_SPLIT, attn_generic=1),
             "fused": dict(attn_bwd=L.ATTN_BWD_FUSED)}[path]
    with L.override(**force):
        o, dq, dkv, do = _grads(q, kv, H, kpm, fused=True)
    rq, rkv = _ref_grads(q, kv, H, kpm, do)
    tol = 5e-5 if dtype == torch.float32 else 3e-2
    close(dq, rq, tol)
    close(dkv, rkv, tol)


@pytest.mark.parametrize("case,masked", [((2, 64, 776, 4, 64), True), ((2, 160, 300, 8, 64), True),
                                         ((1, 300, 701, 2, 64), False), ((1, 5120, 5248, 8, 64), True)])
def test_backward_dq_lds_dma_form(case, masked):
    """The dQ pass's LDS-DMA staging form (override attn_dq_dma = 1: K / V
    blocks and the key-mask bytes by buffer_load ... lds into a 3-deep ring,
    the kimg swizzle undone in the per-lane source offsets) equals the
    register-staged form bit for bit, where the host takes it (kv_len % 4 == 0
    with a mask; any kv_len without), and matches float64."""
    from mtts import _lib as L
    B, T, S, H, hd = case
    q, kv, kpm = make(B, T, S, H, hd, torch.bfloat16, seed=7)
    if not masked:
        kpm = None
    with L.override(attn_bwd=L.ATTN_BWD_SPLIT, attn_dq_dma=0):
        o, dq0, dkv0, do = _grads(q, kv, H, kpm, fused=True)
    with L.override(attn_bwd=L.ATTN_BWD_SPLIT, attn_dq_dma=1):
        o1, dq1, dkv1, do1 = _grads(q, kv, H, kpm, fused=True)
    assert torch.equal(do, do1) and torch.equal(dq0, dq1) and torch.equal(dkv0, dkv1)
    if T * S <= 300 * 1000:
        rq, rkv = _ref_grads(q, kv, H, kpm, do)
        close(dq1, rq, 3e-2)


@pytest.mark.parametrize("hd", [128, 64])
def test_backward_c5_shape_bf16(hd):
    """train.py decoder shape: T_audio = 5120 queries, 5120 reference keys +
    128 text keys, H=8, d = 1024 or train.py's 512 (reference gradients of
    one batch by the full-key float64 restatement)."""
    B, T, S, H = 1, 5120, 5248, 8
    q, kv, kpm = make(B, T, S, H, hd, torch.bfloat16, seed=13)
    o, dq, dkv, do = _grads(q, kv, H, kpm, fused=True)
    assert torch.isfinite(dq).all() and torch.isfinite(dkv).all()
    rq, rkv = _ref_grads(q, kv, H, kpm, do)
    close(dq, rq, 3e-2)
    close(dkv, rkv, 3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_single_query_fully_masked_and_generic_agree(dtype):
    """q_len == 1 (single-query kernel): a fully masked batch row is NaN with
    lse = -inf like torch, other rows match the float64 reference and the
    generic MFMA kernel (override attn_generic) on the same inputs."""
    from mtts import _lib as L
    from mtts import attn_kernels as A
    B, S, H, hd = 4, 77, 8, 128
    q, kv, kpm = make(B, 1, S, H, hd, dtype, seed=3, full_mask_batch=2)
    d = H * hd
    out, lse = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    assert torch.isnan(out[2]).all() and torch.isneginf(lse[2]).all()
    keep = [0, 1, 3]
    ref, ref_lse = ref_attention(q[keep], kv[keep, :, :d], kv[keep, :, d:], H, kpm[keep])
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    close(out[keep], ref, tol)
    close(lse[keep], ref_lse, 1e-5)
    with L.override(attn_generic=1):
        out2, _ = A.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
    close(out[keep], out2[keep].double(), tol)


@pytest.mark.parametrize("B,S,H,hd", [(32, 128, 8, 128), (3, 77, 4, 64), (2, 200, 2, 64)])
def test_decode_head_major_kv_matches_channel_last(B, S, H, hd):
    """Single-query attention reading head-major (B, H, S, hd) K / V copies
    (kv_hs head stride; the decode engine's per-context layout) equals the
    channel-last call bit for bit (same kernel arithmetic)."""
    from mtts.attn_kernels import attention_decode_packed
    g = torch.Generator(device="cpu").manual_seed(B + S + H)
    d = H * hd
    q = torch.randn(B, d, generator=g).to("cuda", torch.bfloat16)
    kv = torch.randn(B, S, 2 * d, generator=g).to("cuda", torch.bfloat16)
    kpm = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    kpm[:, S - 5:] = True
    k, v = kv[..., :d], kv[..., d:]
    a = attention_decode_packed(q, k, v, H, kpm)
    khm = k.reshape(B, S, H, hd).permute(0, 2, 1, 3).contiguous()
    vhm = v.reshape(B, S, H, hd).permute(0, 2, 1, 3).contiguous()
    b = attention_decode_packed(q, khm, vhm, H, kpm)
    assert torch.equal(a.unpack(), b.unpack())


@pytest.mark.parametrize("B,S,H,hd,d", [(32, 128, 8, 128, 1024), (5, 77, 16, 64, 1024), (3, 200, 4, 64, 256)])
def test_decode_qproj_fused_matches_projection_then_attention(B, S, H, hd, d):
    """mtts_attention_decode_qproj (the decode step's LayerNorm + q
    projection inside the single-query attention kernel) against the
    unfused packed path it replaces -- ops.gemm_rows with the LayerNorm
    prologue, then attention_decode_packed -- and against an fp32 torch
    composition.  The q values may round differently by one bf16 ulp (a
    different summation order): 2e-2 of the output scale."""
    from mtts import ops
    from mtts.attn_kernels import attention_decode_packed, attention_decode_qproj_packed
    g = torch.Generator(device="cpu").manual_seed(B + S + H + d)
    x = torch.randn(B, d, generator=g).to("cuda", torch.bfloat16)
    wq = (torch.randn(H * hd, d, generator=g) / d ** 0.5).to("cuda", torch.bfloat16)
    bq = (0.1 * torch.randn(H * hd, generator=g)).to("cuda", torch.bfloat16)
    lnw = (1 + 0.1 * torch.randn(d, generator=g)).cuda()
    lnb = (0.1 * torch.randn(d, generator=g)).cuda()
    kv = torch.randn(B, S, 2 * H * hd, generator=g).to("cuda", torch.bfloat16)
    kpm = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    kpm[:, S - 7:] = True
    dd = H * hd
    khm = kv[..., :dd].reshape(B, S, H, hd).permute(0, 2, 1, 3).contiguous()
    vhm = kv[..., dd:].reshape(B, S, H, hd).permute(0, 2, 1, 3).contiguous()
    fused = attention_decode_qproj_packed(x, wq, bq, lnw, lnb, 1e-5, khm, vhm, H, kpm).unpack().float()
    q = ops.gemm_rows(x, wq, bq, ln=(lnw, lnb, 1e-5, None, None))
    unfused = attention_decode_packed(q, khm, vhm, H, kpm).unpack().float()
    xn = F.layer_norm(x.float(), (d,), lnw, lnb, 1e-5).bfloat16().float()
    qr = (xn @ wq.float().t() + bq.float()).bfloat16()
    ref, _ = ref_attention(qr[:, None], kv[..., :dd], kv[..., dd:], H, kpm)
    close(fused, unfused.double(), 2e-2)
    close(fused, ref[:, 0], 2e-2)
