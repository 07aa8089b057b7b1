"""GPU parity of the drop-in modules (mamba_decoder.py, style_cross_attention.py)
against golden vectors produced by the REFERENCE modules themselves
(tests/golden/make_golden.py), fp32, tolerance 1e-3 relative."""
import numpy as np
import pytest
import torch

from test_gpu_ops import close, DEV

pytestmark = pytest.mark.gpu


def _load(model, g):
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd/")}
    model.load_state_dict(sd)
    return model


def _decoder(golden):
    import mamba_decoder
    g = golden("decoder.npz")
    m = mamba_decoder.MambaTTSDecoder(vocab_size_audio=10, d_model=64, n_layers=2, n_heads=4, d_ff=128,
                                      d_style=16, max_len=256)
    return _load(m, g).to(DEV), g


@pytest.mark.parametrize("tag", ["plain", "masked_ref"])
def test_decoder_forward_backward_vs_reference(golden, tag):
    m, g = _decoder(golden)
    m.train()
    tokens = torch.from_numpy(g["tokens"]).to(DEV)
    text = torch.from_numpy(g["text"]).to(DEV).requires_grad_(True)
    z = torch.from_numpy(g["z_style"]).to(DEV).requires_grad_(True)
    kw = {}
    if tag == "masked_ref":
        ref = torch.from_numpy(g["ref"]).to(DEV).requires_grad_(True)
        kw = dict(text_mask=torch.from_numpy(g["text_mask"]).to(DEV), ref_hidden=ref,
                  ref_mask=torch.from_numpy(g["ref_mask"]).to(DEV))
    logits = m(tokens, text, z, **kw)
    close(logits, g[f"{tag}/logits"], name="logits")
    (logits * torch.from_numpy(g[f"{tag}/G"]).to(DEV)).sum().backward()
    close(text.grad, g[f"{tag}/dtext"], name="dtext")
    close(z.grad, g[f"{tag}/dz"], name="dz")
    if tag == "masked_ref":
        close(kw["ref_hidden"].grad, g[f"{tag}/dref"], name="dref")
    for n, p in m.named_parameters():
        close(p.grad, g[f"{tag}/grad/{n}"], name=n)


def test_decode_step_sequence_vs_reference(golden):
    m, g = _decoder(golden)
    m.eval()
    tokens = torch.from_numpy(g["tokens"]).to(DEV)
    text = torch.from_numpy(g["text"]).to(DEV)
    z = torch.from_numpy(g["z_style"]).to(DEV)
    kw = dict(text_mask=torch.from_numpy(g["text_mask"]).to(DEV), ref_hidden=torch.from_numpy(g["ref"]).to(DEV),
              ref_mask=torch.from_numpy(g["ref_mask"]).to(DEV))
    states = [None, None]
    outs = []
    with torch.no_grad():
        for t in range(g["decode/logits"].shape[1]):
            lg, states = m.decode_step(tokens[:, t:t + 1], text, z, states, t, **kw)
            outs.append(lg)
    close(torch.cat(outs, 1), g["decode/logits"], name="decode logits")
    for i, (cs, ss) in enumerate(states):
        close(cs, g[f"decode/conv_state{i}"], name=f"conv_state{i}")
        close(ss, g[f"decode/ssm_state{i}"], name=f"ssm_state{i}")


def test_decode_steps_equal_teacher_forced_forward(golden):
    """Property: with quant_embed zeroed (decode_step omits it), T decode steps
    reproduce the teacher-forced logits."""
    m, g = _decoder(golden)
    m.eval()
    with torch.no_grad():
        m.quant_embed.weight.zero_()
        tokens = torch.from_numpy(g["tokens"]).to(DEV)[:, :20]
        text = torch.from_numpy(g["text"]).to(DEV)
        z = torch.from_numpy(g["z_style"]).to(DEV)
        full = m(tokens, text, z)
        states = [None, None]
        outs = []
        for t in range(tokens.shape[1]):
            lg, states = m.decode_step(tokens[:, t:t + 1], text, z, states, t)
            outs.append(lg)
    close(torch.cat(outs, 1), full, name="steps vs forward")


def test_fully_masked_row_gives_nan_like_reference(golden):
    m, g = _decoder(golden)
    tokens = torch.from_numpy(g["tokens"]).to(DEV)[:, :8]
    text = torch.from_numpy(g["text"]).to(DEV)
    z = torch.from_numpy(g["z_style"]).to(DEV)
    mask = torch.ones(3, text.shape[1], dtype=torch.bool, device=DEV)
    mask[1] = False  # kpm = ~mask -> row 1 attends to nothing
    with torch.no_grad():
        lg = m(tokens, text, z, text_mask=mask)
    assert torch.isnan(lg[1]).all() and torch.isfinite(lg[0]).all() and torch.isfinite(lg[2]).all()


def test_bf16_decoder_tracks_fp32(golden):
    m, g = _decoder(golden)
    tokens = torch.from_numpy(g["tokens"]).to(DEV)
    text = torch.from_numpy(g["text"]).to(DEV)
    z = torch.from_numpy(g["z_style"]).to(DEV)
    with torch.no_grad():
        ref = m(tokens, text, z)
        m.compute_dtype = torch.bfloat16
        lg = m(tokens, text, z)
    assert lg.dtype == torch.bfloat16
    close(lg.float(), ref, rtol=5e-2, name="bf16 logits")


@pytest.mark.parametrize("graph", [False, True])
def test_bf16_decode_engine_rows_vs_blas(golden, graph, monkeypatch):
    """bf16 engine: the HIP skinny-GEMM projections (csrc/rows.hip) against
    the same engine on hipBLASLt, and both against the fp32 module path."""
    from mtts import ops
    from mtts.decode import DecodeEngine
    calls = []
    real = ops.gemm_rows
    monkeypatch.setattr(ops, "gemm_rows", lambda *a, **k: calls.append(1) or real(*a, **k))
    m, g = _decoder(golden)
    m.eval()
    tokens = torch.from_numpy(g["tokens"]).to(DEV)
    kw = dict(text_mask=torch.from_numpy(g["text_mask"]).to(DEV), ref_hidden=torch.from_numpy(g["ref"]).to(DEV),
              ref_mask=torch.from_numpy(g["ref_mask"]).to(DEV))
    text = torch.from_numpy(g["text"]).to(DEV)
    z = torch.from_numpy(g["z_style"]).to(DEV)
    m.compute_dtype = torch.bfloat16
    outs = []
    for rows in (True, False):
        eng = DecodeEngine(m, use_graph=graph, use_rows=rows)
        states = [None, None]
        seq = []
        with torch.no_grad():
            for t in range(g["decode/logits"].shape[1]):
                lg, states = eng.step(tokens[:, t:t + 1], text, z, states, t, **kw)
                seq.append(lg.float().clone())
        outs.append(torch.cat(seq, 1))
    assert len(calls) >= 6 * 2, "skinny-GEMM path not taken"
    close(outs[0], outs[1], rtol=3e-2, name="rows vs hipBLASLt engine (bf16)")
    close(outs[0], g["decode/logits"], rtol=5e-2, name="bf16 rows engine vs fp32 reference")


def test_style_pipeline_vs_reference(golden):
    import style_cross_attention as sca
    g = golden("style.npz")
    p = sca.StyleConditioningPipeline(d_style=16, d_model=64, num_heads=4, dropout=0.1)
    p = _load(p, g).to(DEV).eval()
    text = torch.from_numpy(g["text"]).to(DEV)
    style = torch.from_numpy(g["style"]).to(DEV)
    dur = torch.from_numpy(g["durations"]).to(DEV)
    with torch.no_grad():
        frames, lengths, K, V = p(text, style, dur)
        fc, lc, _, _ = p(text, style, dur, max_frame_len=7)
    close(frames, g["frames"], name="frames")
    assert torch.equal(lengths.cpu(), torch.from_numpy(g["lengths"]))
    close(K, g["K"], name="K")
    close(V, g["V"], name="V")
    close(fc, g["frames_cap"], name="frames_cap")
    assert torch.equal(lc.cpu(), torch.from_numpy(g["lengths_cap"]))


def test_mamba_ssm_shim_mixer_matches_oracle(golden):
    """`from mamba_ssm import Mamba` (the reference's import line,
    mamba_decoder.py:4) resolves to the HIP mixer, and a mixer built the way
    the reference builds it (`Mamba(d_model, d_state=16, d_conv=4, expand=2)`,
    mamba_decoder.py:26) with layer 0's golden weights computes the oracle's
    mixer (`mamba_forward_ref`, pinned by the golden fixtures) under the
    `(out, state)` contract of mamba_decoder.py:10-15: outputs, both states
    and every input / parameter gradient at 1e-3, fp32.  (The reference file
    itself is not shipped: the decoder goldens above are what it produced.)"""
    import importlib
    import mamba_ssm
    import oracle.mamba_ref as R
    assert mamba_ssm.Mamba.__module__ == "mtts.mamba"
    assert importlib.import_module("mamba_decoder").Mamba is mamba_ssm.Mamba
    g = golden("decoder.npz")
    pre = "sd/layers.0.mamba."
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(pre)}
    mix = mamba_ssm.Mamba(64, d_state=16, d_conv=4, expand=2)
    mix.load_state_dict(sd)
    mix = mix.to(DEV)
    torch.manual_seed(3)
    x = torch.randn(3, 37, 64, dtype=torch.float64)
    G = torch.randn(3, 37, 64, dtype=torch.float64)
    xg = x.float().to(DEV).requires_grad_(True)
    out, (conv_state, ssm_state) = mix(xg)
    (out * G.float().to(DEV)).sum().backward()
    p = {k: v.double().requires_grad_(True) for k, v in sd.items()}
    xr = x.clone().requires_grad_(True)
    ro, (rc, rs) = R.mamba_forward_ref(p, "", xr)
    (ro * G).sum().backward()
    close(out, ro, name="mixer out")
    close(conv_state, rc, name="conv_state")
    close(ssm_state, rs, name="ssm_state")
    close(xg.grad, xr.grad, name="dx")
    for n, t in mix.named_parameters():
        close(t.grad, p[n].grad, name=n)


@pytest.mark.parametrize("mode", ["graph", "eager"])
def test_decode_engine_matches_module_path(golden, mode):
    """The incremental engine (cached K/V + FiLM, in-place states, hipGraph
    replay) equals the generic per-module decode path step by step, and its
    states equal the reference goldens."""
    m, g = _decoder(golden)
    m.eval()
    tokens = torch.from_numpy(g["tokens"]).to(DEV)
    kw = dict(text_mask=torch.from_numpy(g["text_mask"]).to(DEV), ref_hidden=torch.from_numpy(g["ref"]).to(DEV),
              ref_mask=torch.from_numpy(g["ref_mask"]).to(DEV))
    text = torch.from_numpy(g["text"]).to(DEV)
    z = torch.from_numpy(g["z_style"]).to(DEV)
    outs = {}
    for dm in (None, mode):
        m.decode_mode = dm
        m.reset_decode_cache()
        states = [None, None]
        seq = []
        with torch.no_grad():
            for t in range(g["decode/logits"].shape[1]):
                lg, states = m.decode_step(tokens[:, t:t + 1], text, z, states, t, **kw)
                seq.append(lg.clone())
        outs[dm] = (torch.cat(seq, 1), [(a.clone(), b.clone()) for a, b in states])
    close(outs[mode][0], outs[None][0], rtol=1e-5, name="engine logits")
    close(outs[mode][0], g["decode/logits"], name="engine vs reference")
    for i in range(2):
        close(outs[mode][1][i][1], g[f"decode/ssm_state{i}"], name="ssm state")


@pytest.mark.parametrize("B", [32, 5, 33])
def test_bf16_decode_engine_c4_shapes(B):
    """C4-shaped layers (d_model=1024, d_ff=2048, 8 heads; 2 layers): the
    fused engine step (LayerNorm prologues, residual / conv epilogues,
    single-query attention; B <= 32) and its fallback (B = 33: hipBLASLt
    projections) against the generic module path, bf16, several steps.
    Bound: 3e-2 of the logit scale (bf16 roundings of the activations)."""
    import mamba_decoder
    from mtts.decode import DecodeEngine
    torch.manual_seed(1)
    m = mamba_decoder.MambaTTSDecoder(10, d_model=1024, n_layers=2, n_heads=8, d_ff=2048, d_style=256).to(DEV).eval()
    m.compute_dtype = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(2)
    text = torch.randn(B, 40, 1024, device=DEV, generator=g)
    z = torch.randn(B, 256, device=DEV, generator=g)
    mask = torch.ones(B, 40, dtype=torch.bool, device=DEV)
    mask[:, 30:] = False
    tok = torch.randint(0, 10, (B, 1), device=DEV, generator=g)
    outs = []
    for mode in ("engine", "module"):
        m.decode_mode = None
        eng = DecodeEngine(m, use_graph=True) if mode == "engine" else None
        states = [None, None]
        seq = []
        with torch.no_grad():
            for t in range(6):
                if eng is not None:
                    lg, states = eng.step(tok, text, z, states, t, text_mask=mask)
                else:
                    lg, states = m.decode_step(tok, text, z, states, t, text_mask=mask)
                seq.append(lg.float().clone())
        outs.append(torch.cat(seq, 1))
    assert (B <= 32) == DecodeEngine(m)._fused_ok(torch.bfloat16, B)
    close(outs[0], outs[1], rtol=3e-2, name=f"engine vs module path, B={B}")


def test_decode_engine_out_of_range_token_raises():
    """A last_token outside token_embed: the reference's nn.Embedding raises
    (mamba_decoder.py:217).  The fused engine embeds through mtts_embed_sum,
    which zero-fills the row (no uninitialised memory reaches the logits or
    the states) and flags it; the engine reads the flag without a host sync
    and raises IndexError at a later decode_step (best-effort, deferred) or at
    the blocking check_errors(), then clears it (the following steps run
    normally); reset() raises a pending flag, clearing it, so a new session
    starts clean and no error is lost."""
    import mamba_decoder
    torch.manual_seed(1)
    m = mamba_decoder.MambaTTSDecoder(10, d_model=1024, n_layers=2, n_heads=8, d_ff=2048, d_style=256).to(DEV).eval()
    m.compute_dtype = torch.bfloat16
    B = 4
    text = torch.randn(B, 16, 1024, device=DEV)
    z = torch.randn(B, 256, device=DEV)
    good = torch.randint(0, 10, (B, 1), device=DEV)
    bad = good.clone()
    bad[2, 0] = 10
    with torch.no_grad():
        lg, st = m.decode_step(good, text, z, [None, None], 0)
        assert m._engine.fused
        lg, st = m.decode_step(bad, text, z, st, 1)
        assert torch.isfinite(lg).all()
        torch.cuda.synchronize()
        with pytest.raises(IndexError, match="out of range"):
            m.decode_step(good, text, z, st, 2)
        lg, st = m.decode_step(good, text, z, st, 2)
        torch.cuda.synchronize()
        lg, st = m.decode_step(good, text, z, st, 3)
        assert torch.isfinite(lg).all()
        # check_errors() is the blocking guarantee; reset() clears a pending flag
        eng = m._engine
        eng.check_errors()
        m.decode_step(bad, text, z, st, 4)
        with pytest.raises(IndexError, match="out of range"):
            eng.check_errors()
        eng.check_errors()
        m.decode_step(bad, text, z, st, 5)
        with pytest.raises(IndexError, match="out of range"):   # reset() raises a pending flag, then clears it
            eng.reset()
        eng.reset()
        lg, st = m.decode_step(good, text, z, [None, None], 0)
        torch.cuda.synchronize()
        m.decode_step(good, text, z, st, 1)
        eng.check_errors()
