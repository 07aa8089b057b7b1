"""GPU parity at the BASELINE.json configurations and the round-2 contract
fixes.

Config coverage (BASELINE.json configs / SURVEY.md §8d):
  * C1  - 2L d_model=256, B=2, T_audio=128, fp32 fwd+bwd vs the float64 oracle
          decoder (every parameter gradient);
  * C2  - the scan at C2's shape (B=8, d_inner=2048, L=2048; default dispatch:
          one-pass LDS-DMA forward, 4-segment backward with the carry pass),
          fp32 and bf16 I/O, all 8 gradients; a 2-layer d_model=1024 decoder
          at B=8, T=2048 fwd+bwd (fp32 at 1e-3, bf16 at a stated bound);
  * north star - selective_scan fwd at B=32, L=8192, d_inner=2048 (the c1
          kernel) vs the oracle on batch/channel slices at full length;
  * C5  - the train.py shape (5 x 1024 flattened codec streams, 5120
          reference keys + 128 text keys) on a 2-layer d_model=1024 decoder,
          bf16, vs the float64 oracle.
The oracle (oracle/mamba_ref.py) is evaluated in float64 ON THE GPU for the
large shapes (same restatement, same math; a CPU run at these sizes takes
minutes).  Tolerances: 1e-3 of the reference's max |value| per tensor for
fp32 (the north star's bound); bf16 bounds are stated per test.
"""
import math
import re

import pytest
import torch

from test_gpu_ops import close, DEV
from oracle import mamba_ref as R

pytestmark = pytest.mark.gpu


def _decoder(d_model, n_layers, n_heads=8, d_ff=None, d_style=256, vocab=10, num_quantizers=1, seed=0):
    import mamba_decoder
    torch.manual_seed(seed)
    m = mamba_decoder.MambaTTSDecoder(vocab, d_model=d_model, n_layers=n_layers, n_heads=n_heads,
                                      d_ff=d_ff or 2 * d_model, d_style=d_style, num_quantizers=num_quantizers)
    return m.to(DEV)


def _params64(m, device=DEV):
    return {k: v.detach().to(device, torch.float64).requires_grad_(v.dtype.is_floating_point)
            for k, v in m.state_dict().items()}


def _scan_args(B, L, D, dtype, seed):
    """Decoder-like scan inputs (SURVEY §8d distribution): u, z ~ N(0,1),
    raw delta ~ N(0, 0.1^2), delta_bias = softplus^-1(logU[1e-3, 1e-1]),
    A = -exp(A_log) around -[1..16], B, C ~ N(0,1), D ~ N(1, 0.1^2)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    u = torch.randn(B, L, D, device=DEV, generator=g).to(dtype)
    z = torch.randn(B, L, D, device=DEV, generator=g).to(dtype)
    dl = (torch.randn(B, L, D, device=DEV, generator=g) * 0.1).to(dtype)
    Bm = torch.randn(B, L, 16, device=DEV, generator=g).to(dtype)
    Cm = torch.randn(B, L, 16, device=DEV, generator=g).to(dtype)
    A = -torch.arange(1, 17, device=DEV, dtype=torch.float32).repeat(D, 1) * torch.exp(
        torch.randn(D, 16, device=DEV, generator=g) * 0.1)
    Dp = 1 + 0.1 * torch.randn(D, device=DEV, generator=g)
    dt0 = torch.exp(torch.rand(D, device=DEV, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
    bias = dt0 + torch.log(-torch.expm1(-dt0))
    return u, dl, A, Bm, Cm, Dp, z, bias


# --------------------------------------------------------------------------- C2 scan
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_scan_fwd_bwd_c2_shape_vs_oracle(dtype):
    """C2's scan (B=8, L=2048, d_inner=2048) through the default dispatch,
    forward and all 8 gradients vs the float64 oracle's autograd on the same
    (rounded) inputs.  fp32: 1e-3; bf16 I/O: 1e-2 (bf16 output rounding of
    out / du / ddelta / dz; dB, dC, dA, dD, ddelta_bias are fp32 sums)."""
    from mtts import ops
    B, L, D = 8, 2048, 2048
    u, dl, A, Bm, Cm, Dp, z, bias = _scan_args(B, L, D, dtype, 11)
    out, last, ckpt = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True, want_ckpt=True)
    g = torch.Generator(device=DEV).manual_seed(12)
    dout = torch.randn(B, L, D, device=DEV, generator=g).to(dtype)
    du, dd, dz, dB, dC, dA, dD, db, _ = ops.scan_bwd(u, dl, A, Bm, Cm, Dp, z, bias, True, None, ckpt, dout)
    torch.cuda.synchronize()

    cm = lambda t: t.detach().double().transpose(1, 2).contiguous().requires_grad_(True)  # noqa: E731
    ru, rdl, rB, rC, rz = cm(u), cm(dl), cm(Bm), cm(Cm), cm(z)
    rA, rD, rb = (t.detach().double().requires_grad_(True) for t in (A, Dp, bias))
    ref, rlast = R.selective_scan_ref(ru, rdl, rA, rB, rC, rD, rz, rb, True, return_last_state=True)
    (ref * dout.double().transpose(1, 2)).sum().backward()
    tol = 1e-3 if dtype == torch.float32 else 1e-2
    close(out.transpose(1, 2), ref.detach(), rtol=tol, name="out")
    close(last, rlast.detach(), rtol=1e-3, name="last_state")
    for name, got, want, t in (("du", du, ru, tol), ("ddelta", dd, rdl, tol), ("dz", dz, rz, tol),
                               ("dB", dB, rB, 1e-3), ("dC", dC, rC, 1e-3)):
        close(got.transpose(1, 2), want.grad, rtol=t, name=name)
    close(dA, rA.grad, rtol=1e-3, name="dA")
    close(dD, rD.grad, rtol=1e-3, name="dD")
    close(db, rb.grad, rtol=1e-3, name="ddelta_bias")


# --------------------------------------------------------------------------- north star, full L
def test_scan_north_star_full_length_slices():
    """The roofline kernel's own shape (B=32, L=8192, d_inner=2048, fp32 I/O,
    softplus + z gate): every one of the 8192 steps of 4 batch rows x 128
    channels (two 64-channel waves each, at both ends of the channel range)
    vs the float64 oracle, plus the last state; fp32 1e-3."""
    from mtts import ops
    B, L, D = 32, 8192, 2048
    u, dl, A, Bm, Cm, Dp, z, bias = _scan_args(B, L, D, torch.float32, 21)
    out, last, _ = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True)
    torch.cuda.synchronize()
    bs = [0, 9, 22, 31]
    cs = torch.cat([torch.arange(0, 64), torch.arange(D - 64, D)]).to(DEV)
    sl = lambda t: t[bs][:, :, cs].double().transpose(1, 2)  # noqa: E731
    bc = lambda t: t[bs].double().transpose(1, 2)  # noqa: E731
    with torch.no_grad():
        ref, rlast = R.selective_scan_ref(sl(u), sl(dl), A[cs].double(), bc(Bm), bc(Cm), Dp[cs].double(), sl(z),
                                          bias[cs].double(), True, return_last_state=True)
    close(out[bs][:, :, cs].transpose(1, 2), ref, name="north-star out slices")
    close(last[bs][:, cs], rlast, name="north-star last_state slices")
    # the rest of the tensor: finite, and every (b, d) row moved (no skipped waves)
    assert torch.isfinite(out).all()
    assert (out.abs().amax(1) > 0).all()


# --------------------------------------------------------------------------- C1
def test_c1_decoder_fwd_bwd_vs_oracle():
    """C1 (BASELINE configs[0]): 2 layers, d_model=256 (8 heads, d_ff 2048,
    d_style 256: the reference defaults), B=2, T_audio=128, 16 text keys with
    padding, fp32: logits and every gradient vs the float64 oracle, 1e-3."""
    m = _decoder(256, 2, d_ff=2048)
    m.train()
    g = torch.Generator().manual_seed(3)
    B, T, Tt = 2, 128, 16
    tok = torch.randint(0, 10, (B, T), generator=g)
    text = torch.randn(B, Tt, 256, generator=g)
    z = torch.randn(B, 256, generator=g)
    mask = torch.ones(B, Tt, dtype=torch.bool)
    mask[1, 11:] = False
    G = torch.randn(B, T, 10, generator=g)
    th = text.to(DEV).requires_grad_(True)
    zz = z.to(DEV).requires_grad_(True)
    logits = m(tok.to(DEV), th, zz, text_mask=mask.to(DEV))
    (logits * G.to(DEV)).sum().backward()
    p = _params64(m, "cpu")
    t64, z64 = text.double().requires_grad_(True), z.double().requires_grad_(True)
    ref = R.decoder_forward_ref(p, 2, 8, tok, t64, z64, text_mask=mask)
    (ref * G.double()).sum().backward()
    close(logits, ref.detach(), name="C1 logits")
    close(th.grad, t64.grad, name="C1 dtext")
    close(zz.grad, z64.grad, name="C1 dz_style")
    for n, prm in m.named_parameters():
        close(prm.grad, p[n].grad, name=f"C1 d{n}")


def _rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


# --------------------------------------------------------------------------- C2 decoder
# bf16 (the bench's precision: bf16 activations, bf16 operands on the
# hand-written NT / TN / skinny GEMMs, fused FFN epilogues, bf16 scan I/O)
# against the float64 oracle at C2's layer shape.  Measured errors (relative to
# the reference's max |value|, MI355X, this seed) -> bound = 3x measured;
# keys are the gradient names with the layer index dropped (max over the two
# layers).  Measured in round 4 (profiles/r04_c2_bf16_errors.txt).
C2_BF16_MEASURED = {
    "logits": 5.30e-03,
    "dtext": 7.41e-03,
    "dtoken_embed.weight": 6.00e-03,
    "dpos_embed.weight": 7.14e-03,
    "dquant_embed.weight": 5.49e-03,
    "dlayers.norm_mamba.weight": 6.40e-03,
    "dlayers.norm_mamba.bias": 7.47e-03,
    "dlayers.mamba.A_log": 7.36e-03,
    "dlayers.mamba.D": 9.54e-03,
    "dlayers.mamba.in_proj.weight": 6.18e-03,
    "dlayers.mamba.conv1d.weight": 1.00e-02,
    "dlayers.mamba.conv1d.bias": 7.55e-03,
    "dlayers.mamba.x_proj.weight": 1.74e-02,
    "dlayers.mamba.dt_proj.weight": 1.46e-02,
    "dlayers.mamba.dt_proj.bias": 1.14e-02,
    "dlayers.mamba.out_proj.weight": 8.53e-03,
    "dlayers.norm_cross.weight": 1.15e-02,
    "dlayers.norm_cross.bias": 6.67e-03,
    "dlayers.cross_attn.in_proj_weight": 4.83e-03,
    "dlayers.cross_attn.in_proj_bias": 4.34e-03,
    "dlayers.cross_attn.out_proj.weight": 5.12e-03,
    "dlayers.cross_attn.out_proj.bias": 4.76e-03,
    "dlayers.norm_ff.weight": 7.91e-03,
    "dlayers.norm_ff.bias": 4.72e-03,
    "dlayers.ff.0.weight": 5.50e-03,
    "dlayers.ff.0.bias": 5.17e-03,
    "dlayers.ff.2.weight": 6.04e-03,
    "dlayers.ff.2.bias": 4.59e-03,
    "dlayers.style_mlp.0.weight": 6.14e-03,
    "dlayers.style_mlp.0.bias": 5.16e-03,
    "dnorm_out.weight": 2.51e-03,
    "dnorm_out.bias": 3.51e-03,
    "dhead.weight": 5.14e-03,
    "dhead.bias": 1.14e-03}
C2_BF16_BOUNDS = {   # 3x measured, rounded down to 2 significant digits
    "logits": 0.015,
    "dtext": 0.022,
    "dtoken_embed.weight": 0.018,
    "dpos_embed.weight": 0.021,
    "dquant_embed.weight": 0.016,
    "dlayers.norm_mamba.weight": 0.019,
    "dlayers.norm_mamba.bias": 0.022,
    "dlayers.mamba.A_log": 0.022,
    "dlayers.mamba.D": 0.028,
    "dlayers.mamba.in_proj.weight": 0.018,
    "dlayers.mamba.conv1d.weight": 0.03,
    "dlayers.mamba.conv1d.bias": 0.022,
    "dlayers.mamba.x_proj.weight": 0.052,
    "dlayers.mamba.dt_proj.weight": 0.043,
    "dlayers.mamba.dt_proj.bias": 0.034,
    "dlayers.mamba.out_proj.weight": 0.025,
    "dlayers.norm_cross.weight": 0.034,
    "dlayers.norm_cross.bias": 0.02,
    "dlayers.cross_attn.in_proj_weight": 0.014,
    "dlayers.cross_attn.in_proj_bias": 0.013,
    "dlayers.cross_attn.out_proj.weight": 0.015,
    "dlayers.cross_attn.out_proj.bias": 0.014,
    "dlayers.norm_ff.weight": 0.023,
    "dlayers.norm_ff.bias": 0.014,
    "dlayers.ff.0.weight": 0.016,
    "dlayers.ff.0.bias": 0.015,
    "dlayers.ff.2.weight": 0.018,
    "dlayers.ff.2.bias": 0.013,
    "dlayers.style_mlp.0.weight": 0.018,
    "dlayers.style_mlp.0.bias": 0.015,
    "dnorm_out.weight": 0.0075,
    "dnorm_out.bias": 0.01,
    "dhead.weight": 0.015,
    "dhead.bias": 0.0034}


def _c2_bound(name):
    return C2_BF16_BOUNDS.get(re.sub(r"^dlayers\.\d+\.", "dlayers.", name))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_c2_shape_two_layer_decoder_vs_oracle(dtype):
    """C2's layer shape (d_model=1024, 8 heads, d_ff 2048, d_style 256) and
    batch (B=8, T_audio=2048, 128 text keys, 10 % padded) on 2 layers, fwd +
    bwd vs the float64 oracle (evaluated on the GPU).  fp32: logits, input
    and every parameter gradient at 1e-3.  bf16 (compute_dtype, the bench's
    precision, i.e. the path bench.py times): every tensor's measured error is
    printed, and bounded by 3x its measured value (C2_BF16_BOUNDS)."""
    from mtts import linear as LIN
    m = _decoder(1024, 2, d_ff=2048)
    m.train()
    if dtype == torch.bfloat16:
        m.compute_dtype = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(5)
    B, T, Tt = 8, 2048, 128
    tok = torch.randint(0, 10, (B, T), device=DEV, generator=g)
    text = torch.randn(B, Tt, 1024, device=DEV, generator=g)
    z = torch.randn(B, 256, device=DEV, generator=g)
    mask = torch.ones(B, Tt, dtype=torch.bool, device=DEV)
    mask[:, int(Tt * 0.9):] = False
    G = torch.randn(B, T, 10, device=DEV, generator=g)
    th = text.clone().requires_grad_(True)
    routed = []
    real_route = LIN._nt_route
    LIN._nt_route = lambda *a, **k: routed.append(real_route(*a, **k)) or routed[-1]
    try:
        logits = m(tok, th, z, text_mask=mask)
        (logits.float() * G).sum().backward()
    finally:
        LIN._nt_route = real_route
    torch.cuda.synchronize()
    if dtype == torch.bfloat16:
        assert any(routed), "the bf16 C2 projections must run on the hand-written NT kernel"
    p = _params64(m)
    t64 = text.double().requires_grad_(True)
    ref = R.decoder_forward_ref(p, 2, 8, tok, t64, z.double(), text_mask=mask)
    (ref * G.double()).sum().backward()
    if dtype == torch.float32:
        close(logits.float(), ref.detach(), rtol=1e-3, name="C2 logits")
        close(th.grad, t64.grad, rtol=1e-3, name="C2 dtext")
        for n, prm in m.named_parameters():
            close(prm.grad, p[n].grad, rtol=1e-3, name=f"C2 d{n}")
        return
    errs = {"logits": _rel_err(logits.float(), ref.detach()), "dtext": _rel_err(th.grad, t64.grad)}
    for n, prm in m.named_parameters():
        errs["d" + n] = _rel_err(prm.grad, p[n].grad)
    print("C2 bf16 measured errors (of max|ref|): " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    bad = []
    for k, e in errs.items():
        b = _c2_bound(k)
        assert b is not None, f"no stated bound for {k}"
        if not e <= b:
            bad.append(f"{k}: {e:.3e} > {b:.1e}")
    assert not bad, "; ".join(bad)


# --------------------------------------------------------------------------- C5
# Measured errors of the C5 decoder test below (relative to the reference's
# max |value|, MI355X, this seed; layer index dropped, max over the two
# layers) -> bound = 3x measured.  Measured in round 5
# (profiles/r05_c5_parity_measured_errors.txt).
C5_BF16_MEASURED = {
    "loss": 7.57e-05,
    "logits": 7.01e-03,
    "dtoken_embed.weight": 2.78e-03,
    "dpos_embed.weight": 4.44e-03,
    "dquant_embed.weight": 3.28e-03,
    "dlayers.norm_mamba.weight": 3.78e-03,
    "dlayers.norm_mamba.bias": 3.71e-03,
    "dlayers.mamba.A_log": 5.65e-03,
    "dlayers.mamba.D": 4.54e-03,
    "dlayers.mamba.in_proj.weight": 3.52e-03,
    "dlayers.mamba.conv1d.weight": 3.95e-03,
    "dlayers.mamba.conv1d.bias": 3.70e-03,
    "dlayers.mamba.x_proj.weight": 1.48e-02,
    "dlayers.mamba.dt_proj.weight": 5.44e-03,
    "dlayers.mamba.dt_proj.bias": 5.58e-03,
    "dlayers.mamba.out_proj.weight": 3.53e-03,
    "dlayers.norm_cross.weight": 4.43e-03,
    "dlayers.norm_cross.bias": 3.62e-03,
    "dlayers.cross_attn.in_proj_weight": 3.71e-03,
    "dlayers.cross_attn.in_proj_bias": 3.39e-03,
    "dlayers.cross_attn.out_proj.weight": 3.45e-03,
    "dlayers.cross_attn.out_proj.bias": 3.40e-03,
    "dlayers.norm_ff.weight": 3.36e-03,
    "dlayers.norm_ff.bias": 3.71e-03,
    "dlayers.ff.0.weight": 2.57e-03,
    "dlayers.ff.0.bias": 2.58e-03,
    "dlayers.ff.2.weight": 3.14e-03,
    "dlayers.ff.2.bias": 3.25e-03,
    "dlayers.style_mlp.0.weight": 4.33e-03,
    "dlayers.style_mlp.0.bias": 4.33e-03,
    "dnorm_out.weight": 2.06e-03,
    "dnorm_out.bias": 2.86e-03,
    "dhead.weight": 1.36e-03,
    "dhead.bias": 1.81e-03}
C5_BF16_BOUNDS = {   # 3x measured, rounded down to 2 significant digits
    "loss": 0.00022,
    "logits": 0.021,
    "dtoken_embed.weight": 0.0083,
    "dpos_embed.weight": 0.013,
    "dquant_embed.weight": 0.0098,
    "dlayers.norm_mamba.weight": 0.011,
    "dlayers.norm_mamba.bias": 0.011,
    "dlayers.mamba.A_log": 0.016,
    "dlayers.mamba.D": 0.013,
    "dlayers.mamba.in_proj.weight": 0.01,
    "dlayers.mamba.conv1d.weight": 0.011,
    "dlayers.mamba.conv1d.bias": 0.011,
    "dlayers.mamba.x_proj.weight": 0.044,
    "dlayers.mamba.dt_proj.weight": 0.016,
    "dlayers.mamba.dt_proj.bias": 0.016,
    "dlayers.mamba.out_proj.weight": 0.01,
    "dlayers.norm_cross.weight": 0.013,
    "dlayers.norm_cross.bias": 0.01,
    "dlayers.cross_attn.in_proj_weight": 0.011,
    "dlayers.cross_attn.in_proj_bias": 0.01,
    "dlayers.cross_attn.out_proj.weight": 0.01,
    "dlayers.cross_attn.out_proj.bias": 0.01,
    "dlayers.norm_ff.weight": 0.01,
    "dlayers.norm_ff.bias": 0.011,
    "dlayers.ff.0.weight": 0.0077,
    "dlayers.ff.0.bias": 0.0077,
    "dlayers.ff.2.weight": 0.0094,
    "dlayers.ff.2.bias": 0.0097,
    "dlayers.style_mlp.0.weight": 0.012,
    "dlayers.style_mlp.0.bias": 0.012,
    "dnorm_out.weight": 0.0061,
    "dnorm_out.bias": 0.0085,
    "dhead.weight": 0.004,
    "dhead.bias": 0.0054}


def test_c5_train_shape_two_layer_decoder_bf16():
    """train.py's decoder call (configs[4]'s shape): 5 FACodec streams of 1024
    frames flattened to T_audio=5120, the voice prompt embedded through the
    decoder's tables as 5120 reference keys in front of 128 text keys
    (T_kv=5248), codec_ce_loss, backward; 2 layers of d_model=1024, bf16,
    B=1.  vs the float64 oracle: the loss, the logits and EVERY parameter
    gradient, each bounded by 3x its measured error (C5_BF16_BOUNDS)."""
    import codec_tokens as ct
    m = _decoder(1024, 2, d_ff=2048, num_quantizers=5)
    m.compute_dtype = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(8)
    B, Q, Tf, Tt = 1, 5, 1024, 128
    codec = torch.randint(0, 10, (B, Tf, Q), device=DEV, generator=g)
    voice = torch.randint(0, 10, (B, Tf, Q), device=DEV, generator=g)
    text = torch.randn(B, Tt, 1024, device=DEV, generator=g)
    z = torch.randn(B, 256, device=DEV, generator=g)
    tmask = torch.ones(B, Tt, dtype=torch.bool, device=DEV)
    audio, _, _ = ct.flatten_codec_tokens(codec)
    _, v3, _ = ct.flatten_codec_tokens(voice)
    ref_h, vmask = ct.embed_codec_tokens(v3, m)
    logits = m(audio, text, z, text_mask=tmask, ref_hidden=ref_h, ref_mask=vmask)
    loss = ct.codec_ce_loss(logits, audio)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(logits).all() and torch.isfinite(loss)
    p = _params64(m)
    r_ref, r_mask = R.embed_codec_tokens_ref(v3, p["token_embed.weight"], p["pos_embed.weight"],
                                             p["quant_embed.weight"])
    assert torch.equal(r_mask, vmask)
    r_logits = R.decoder_forward_ref(p, 2, 8, audio, text.double(), z.double(), text_mask=tmask,
                                     ref_hidden=r_ref, ref_mask=r_mask)
    r_loss = R.codec_ce_loss_ref(r_logits, audio)
    r_loss.backward()
    errs = {"loss": _rel_err(loss, r_loss.detach()), "logits": _rel_err(logits.float(), r_logits.detach())}
    for n, prm in m.named_parameters():
        k = "d" + re.sub(r"^layers\.\d+\.", "layers.", n)
        errs[k] = max(errs.get(k, 0.0), _rel_err(prm.grad, p[n].grad))
    print("C5 bf16 measured errors (of max|ref|): " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    bad = [f"{k}: {e:.3e} > {C5_BF16_BOUNDS.get(k)}" for k, e in errs.items()
           if C5_BF16_BOUNDS.get(k) is None or not e <= C5_BF16_BOUNDS[k]]
    assert not bad, "; ".join(bad)


# --------------------------------------------------------------------------- contract fixes
def test_3d_tokens_multi_quantizer_raise_like_reference():
    """Quirk 3 (mamba_decoder.py:128-133, 169-171): 3D tokens (B, Q, T) with
    Q > 1 reach `tok (B, Q*T, d) + pos (B, T, d)` and raise; Q = 1 works and
    equals the 2D call."""
    m = _decoder(64, 1, n_heads=4, d_ff=128, d_style=16, num_quantizers=2)
    tok3 = torch.randint(0, 10, (2, 2, 16), device=DEV)
    text = torch.randn(2, 5, 64, device=DEV)
    z = torch.randn(2, 16, device=DEV)
    with pytest.raises(RuntimeError, match="must match the size"):
        m(tok3, text, z)
    with torch.no_grad():
        a = m(tok3[:, :1], text, z)
        b = m(tok3[:, 0], text, z)
    assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["graph", "eager"])
def test_decode_context_cache_not_stale_after_free(mode):
    """A new conditioning tensor that the caching allocator places at a freed
    tensor's address (same shape, version 0) must not reuse the cached K/V /
    FiLM: decode with utterance A, free it, decode with B, compare with the
    float64 oracle's decode_step on B."""
    m = _decoder(64, 2, n_heads=4, d_ff=128, d_style=16)
    m.eval()
    m.decode_mode = mode
    B, Tt = 2, 12
    z = torch.randn(B, 16, device=DEV)
    tok = torch.randint(0, 10, (B, 1), device=DEV)

    def utterance(seed):
        text = torch.randn(B, Tt, 64, device=DEV, generator=torch.Generator(device=DEV).manual_seed(seed))
        states = [None, None]
        outs = []
        with torch.no_grad():
            for t in range(3):
                lg, states = m.decode_step(tok, text, z, states, t)
                outs.append(lg.clone())
        return text.clone(), torch.cat(outs, 1)

    utterance(100)                      # utterance A's text is dropped by the caller here
    text_b, got_b = utterance(200)
    p = _params64(m)
    st = None
    ref = []
    for t in range(3):
        lg, st = R.decode_step_ref(p, 2, 4, tok, text_b.double(), z.double(), st, t)
        ref.append(lg)
    close(got_b, torch.cat(ref, 1).detach(), name="decode after context switch")


def test_mamba_with_state_backward_vs_oracle():
    """mamba(x, state) with L > 1 under autograd (prefill continued from a
    given conv window and SSM state): outputs and the gradients of x, every
    mixer parameter, conv_state and ssm_state vs the float64 oracle."""
    from mtts.mamba import Mamba
    torch.manual_seed(4)
    mm = Mamba(64).to(DEV)
    B, L = 2, 37
    x = torch.randn(B, L, 64, device=DEV, requires_grad=True)
    cs = (torch.randn(B, 128, 4, device=DEV) * 0.5).requires_grad_(True)
    ss = (torch.randn(B, 128, 16, device=DEV) * 0.5).requires_grad_(True)
    out, (ncs, nss) = mm(x, (cs, ss))
    G = torch.randn_like(out)
    (out * G).sum().backward()
    p = {k: v.detach().double().cpu().requires_grad_(True) for k, v in mm.state_dict().items()}
    x64 = x.detach().double().cpu().requires_grad_(True)
    cs64 = cs.detach().double().cpu().requires_grad_(True)
    ss64 = ss.detach().double().cpu().requires_grad_(True)
    ref, (rcs, rss) = R.mamba_forward_ref(p, "", x64, (cs64, ss64))
    (ref * G.double().cpu()).sum().backward()
    close(out, ref.detach(), name="out")
    close(ncs, rcs.detach(), name="conv_state out")
    close(nss, rss.detach(), name="ssm_state out")
    close(x.grad, x64.grad, name="dx")
    close(cs.grad, cs64.grad, name="d conv_state")
    close(ss.grad, ss64.grad, name="d ssm_state")
    for n, prm in mm.named_parameters():
        close(prm.grad, p[n].grad, name=f"d{n}")


def test_fused_adam_load_state_dict_then_step():
    """FusedClipAdam: step, load_state_dict (new moment tensors), step again
    equals torch.optim.Adam + clip_grad_norm_ doing the same (float64 check of
    the fp32 results at 1e-5)."""
    from mtts.optim import FusedClipAdam
    torch.manual_seed(0)
    ps = [torch.randn(n, device=DEV, requires_grad=True) for n in (1000, 37, 4096)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    opt = FusedClipAdam(ps, lr=1e-2, max_grad_norm=0.5)
    ref = torch.optim.Adam(qs, lr=1e-2)
    grads = [[torch.randn_like(p) for p in ps] for _ in range(3)]

    def step(o, params, gs, clip):
        for p, gg in zip(params, gs):
            p.grad = gg.clone()
        if clip:
            torch.nn.utils.clip_grad_norm_(params, 0.5)
        o.step()

    step(opt, ps, grads[0], False)
    step(ref, qs, grads[0], True)
    sd = opt.state_dict()
    opt2 = FusedClipAdam(ps, lr=1e-2, max_grad_norm=0.5)
    step(opt2, ps, grads[1], False)      # its own first step builds plans on fresh state ...
    opt2.load_state_dict(sd)              # ... which the load replaces (the hazard)
    with torch.no_grad():                 # rewind the parameters to where sd was taken
        for p, q in zip(ps, qs):
            p.copy_(q)
    step(opt2, ps, grads[2], False)
    step(ref, qs, grads[2], True)
    for p, q in zip(ps, qs):
        close(p, q, rtol=1e-5, name="param after load_state_dict + step")


# --------------------------------------------------------------------------- C4
def test_c4_decode_4096_steps_vs_teacher_forced():
    """C4 (BASELINE configs[3]): the 12-layer d_model=1024 decoder, B=32, a
    4096-step decode_step loop on the hipGraph engine (bf16, the bench's
    mode), fed a fixed token sequence, against (1) the teacher-forced bf16
    forward of the same sequence and (2) the float64 oracle forward of two
    of its rows, both with quant_embed zeroed: decode_step adds no quantizer
    embedding (quirk 2, mamba_decoder.py:217-221), so with that row zero the
    two paths compute the same function at every position.  Checked at
    positions 0..3, 100, 1000, 2047, 3000, 4094, 4095: logits within 2e-2
    (engine vs bf16 forward; measured 7.6e-3) and 3e-2 (vs float64; measured
    1.0e-2) of the logit scale, i.e. no drift of the SSM / conv states over
    4096 steps; every state finite at step 4095."""
    m = _decoder(1024, 12, d_ff=2048).eval()
    m.compute_dtype = torch.bfloat16
    with torch.no_grad():
        m.quant_embed.weight.zero_()
    g = torch.Generator(device=DEV).manual_seed(11)
    B, T, Tt = 32, 4096, 128
    tok = torch.randint(0, 10, (B, T), device=DEV, generator=g)
    text = torch.randn(B, Tt, 1024, device=DEV, generator=g)
    z = torch.randn(B, 256, device=DEV, generator=g)
    mask = torch.ones(B, Tt, dtype=torch.bool, device=DEV)
    mask[:, int(Tt * 0.9):] = False
    mask[5, 40:] = False
    out = torch.empty(B, T, 10, device=DEV, dtype=torch.float32)
    states = [None] * 12
    with torch.no_grad():
        for t in range(T):
            lg, states = m.decode_step(tok[:, t:t + 1], text, z, states, t, text_mask=mask)
            out[:, t] = lg[:, 0].float()
        tf = m(tok, text, z, text_mask=mask).float()
    assert m.decode_mode == "graph" and m._engine is not None and m._engine.graph is not None
    for i, (cs, ss) in enumerate(states):
        assert torch.isfinite(cs).all() and torch.isfinite(ss).all(), f"layer {i} state at step 4095"
    steps = [0, 1, 2, 3, 100, 1000, 2047, 3000, 4094, 4095]
    e_tf = _rel_err(out[:, steps], tf[:, steps])
    print(f"C4 engine vs teacher-forced bf16: {e_tf:.3e} of the logit scale")
    assert e_tf <= 2e-2, e_tf
    rows = [0, 5]
    p = _params64(m)
    with torch.no_grad():
        ref = R.decoder_forward_ref(p, 12, 8, tok[rows], text[rows].double(), z[rows].double(), text_mask=mask[rows])
    e_ref = _rel_err(out[rows][:, steps], ref[:, steps])
    print(f"C4 engine vs float64 oracle: {e_ref:.3e} of the logit scale")
    assert e_ref <= 3e-2, e_ref
