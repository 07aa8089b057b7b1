"""GPU parity of the codec-token plumbing: the HIP
embedding sum (decoder prologue, mamba_decoder.py:167-171; reference-voice
embedding, train.py:115-131) against torch's F.embedding autograd / the
oracle restatement, and the train.py helpers (codec_ce_loss,
flatten_codec_tokens, embed_codec_tokens) end to end with the decoder.
fp32: 1e-5 relative (the sum of three fp32 rows is exact up to order);
bf16 output: the bf16 rounding of the fp32 sum, exactly."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_ops import close, DEV
from oracle import mamba_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("vocab", [10, 300])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_embed_sum_prologue_vs_torch(vocab, out_dtype):
    from mtts.embed import embed_sum, check_errors
    g = torch.Generator().manual_seed(vocab)
    B, T, d, Q, P = 3, 37, 64, 4, 64
    tok = torch.randint(0, vocab, (B, T), generator=g)
    qid = torch.randint(0, Q, (T,), generator=g)
    ws = [torch.randn(n, d, generator=g) for n in (vocab, Q, P)]
    dy = torch.randn(B, T, d, generator=g)
    gw = [w.to(DEV).requires_grad_(True) for w in ws]
    x = embed_sum(tok.to(DEV), qid.to(DEV), *gw, out_dtype)
    x.backward(dy.to(DEV, out_dtype))
    check_errors()
    cw = [w.clone().requires_grad_(True) for w in ws]
    ref = F.embedding(tok, cw[0]) + F.embedding(qid, cw[1])[None] + F.embedding(torch.arange(T), cw[2])[None]
    if out_dtype == torch.float32:
        close(x, ref.detach(), rtol=1e-6, name="x")
    else:
        assert torch.equal(x.cpu(), ref.detach().to(torch.bfloat16))
    ref.backward(dy.to(out_dtype).float())
    for a, b, n in zip(gw, cw, ("tok", "quant", "pos")):
        close(a.grad, b.grad, rtol=1e-5, name=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("vocab,n,d", [(10, 40960, 512), (16, 1000, 64), (1, 77, 8), (10, 0, 64)])
def test_embed_table_grad_kernel(dtype, vocab, n, d):
    """mtts_embed_table_grad (the codec vocabulary's token-table gradient):
    per-id row sums of g in fp32 against float64, from a row-strided g; an id
    outside [0, vocab) adds nothing; two calls are bit-identical."""
    from mtts.embed import _table_grad
    g = torch.Generator(device=DEV).manual_seed(n + vocab)
    ids = torch.randint(0, vocab, (n,), device=DEV, generator=g)
    if n > 3:
        ids[3] = vocab          # out of range: skipped (the forward flags it)
    big = torch.randn(n, d + 8, device=DEV, generator=g).to(dtype)
    gr = big[:, :d]
    out = _table_grad(ids, gr, vocab)
    ref = torch.zeros(vocab, d, dtype=torch.float64, device=DEV)
    ok = ids < vocab
    ref.index_add_(0, ids[ok], gr[ok].double())
    assert out.dtype == torch.float32 and out.shape == (vocab, d)
    close(out, ref, rtol=1e-5, name="table grad")
    assert torch.equal(out, _table_grad(ids, gr, vocab))


def test_embed_sum_flags_out_of_range_ids():
    from mtts.embed import embed_sum, check_errors
    w = [torch.randn(n, 8, device=DEV) for n in (10, 1, 16)]
    embed_sum(torch.full((1, 4), 10, device=DEV), torch.zeros(4, device=DEV, dtype=torch.long), *w, torch.float32)
    with pytest.raises(IndexError, match="out of range"):
        check_errors()


@pytest.mark.parametrize("Q,T", [(5, 64), (1, 7), (3, 129)])
def test_embed_codec_tokens_vs_reference(Q, T):
    """codec_tokens.embed_codec_tokens (HIP) vs the oracle restatement of
    train.py:115-131, values, pad mask and gradients into the decoder's
    token / position / quantizer tables."""
    import mamba_decoder
    import codec_tokens as ct
    torch.manual_seed(0)
    dec = mamba_decoder.MambaTTSDecoder(vocab_size_audio=10, d_model=64, n_layers=1, n_heads=4, d_ff=128,
                                        d_style=16, max_len=256, num_quantizers=5).to(DEV)
    tok3 = torch.randint(0, 10, (2, Q, T))
    ref_hidden, mask = ct.embed_codec_tokens(tok3.to(DEV), dec)
    w = torch.randn(ref_hidden.shape)
    (ref_hidden * w.to(DEV)).sum().backward()
    tw, pw, qw = (t.detach().cpu().double().requires_grad_(True) for t in
                  (dec.token_embed.weight, dec.pos_embed.weight, dec.quant_embed.weight))
    r, m = R.embed_codec_tokens_ref(tok3, tw, pw, qw)
    close(ref_hidden, r.detach(), rtol=1e-6, name="ref_hidden")
    assert torch.equal(mask.cpu(), m)
    (r * w.double()).sum().backward()
    close(dec.token_embed.weight.grad, tw.grad, rtol=1e-5, name="d_tok")
    close(dec.pos_embed.weight.grad, pw.grad, rtol=1e-5, name="d_pos")
    close(dec.quant_embed.weight.grad, qw.grad, rtol=1e-5, name="d_quant")


def test_train_step_helpers_end_to_end():
    """The train.py decoder call with the voice prompt as reference
    (flatten -> embed_codec_tokens -> decoder(ref_hidden, ref_mask) ->
    codec_ce_loss -> backward) against the oracle decoder in float64."""
    import mamba_decoder
    import codec_tokens as ct
    torch.manual_seed(0)
    dec = mamba_decoder.MambaTTSDecoder(vocab_size_audio=10, d_model=64, n_layers=2, n_heads=4, d_ff=128,
                                        d_style=16, max_len=256, num_quantizers=5).to(DEV)
    B, T, C, Tref, Tt = 2, 24, 5, 12, 9
    codec = torch.randint(0, 10, (B, T, C))
    voice = torch.randint(0, 10, (B, Tref, C))
    text = torch.randn(B, Tt, 64)
    z = torch.randn(B, 16)
    tmask = torch.ones(B, Tt, dtype=torch.bool)
    tmask[1, 6:] = False
    audio, _, _ = ct.flatten_codec_tokens(codec.to(DEV))
    _, v3, _ = ct.flatten_codec_tokens(voice.to(DEV))
    ref_hidden, vmask = ct.embed_codec_tokens(v3, dec)
    logits = dec(audio, text.to(DEV), z.to(DEV), text_mask=tmask.to(DEV), ref_hidden=ref_hidden, ref_mask=vmask)
    loss = ct.codec_ce_loss(logits, audio)
    loss.backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in dec.state_dict().items()}
    a3 = codec.permute(0, 2, 1).reshape(B, -1)
    r_ref, r_mask = R.embed_codec_tokens_ref(voice.permute(0, 2, 1), p["token_embed.weight"], p["pos_embed.weight"],
                                             p["quant_embed.weight"])
    lg = R.decoder_forward_ref(p, 2, 4, a3, text.double(), z.double(), text_mask=tmask, ref_hidden=r_ref,
                               ref_mask=r_mask)
    lref = R.codec_ce_loss_ref(lg, a3)
    close(logits, lg.detach(), name="logits")
    close(loss, lref.detach(), name="loss")
    lref.backward()
    for k in ("token_embed.weight", "pos_embed.weight", "quant_embed.weight", "layers.0.mamba.in_proj.weight",
              "layers.1.cross_attn.in_proj_weight"):
        close(dict(dec.named_parameters())[k].grad, p[k].grad, name=k)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,V", [(16384, 10), (37, 1024), (5, 3)])
def test_cross_entropy_kernel_matches_torch(rows, V, dtype):
    """mtts.loss.cross_entropy (csrc/loss.hip) = F.cross_entropy(logits.float(),
    targets, ignore_index=0) (train.py:31-42): loss and logits gradient
    (mean over the non-ignored rows), fp32 at 1e-5 relative; all-ignored
    batches give NaN like torch."""
    from mtts.loss import cross_entropy
    g = torch.Generator(device="cpu").manual_seed(rows + V)
    x = (torch.randn(rows, V, generator=g) * 3).to("cuda", dtype).requires_grad_(True)
    t = torch.randint(0, V, (rows,), generator=g).to("cuda")
    loss = cross_entropy(x, t, ignore_index=0)
    (loss * 0.7).backward()
    xr = x.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr, t, ignore_index=0)
    (ref * 0.7).backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item()) + 1e-6
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    err = (x.grad.float() - xr.grad).abs().max().item()
    assert err <= tol * xr.grad.abs().max().item() + 1e-8, err
    z = cross_entropy(x.detach(), torch.zeros_like(t), ignore_index=0)
    assert torch.isnan(z)


def test_codec_ce_loss_uses_hip_kernel():
    """codec_ce_loss (train.py:31-42 drop-in) runs csrc/loss.hip and equals
    the reference formula on a (B, T, V) batch with padding."""
    import codec_tokens
    g = torch.Generator(device="cpu").manual_seed(3)
    logits = torch.randn(2, 50, 10, generator=g).to("cuda", torch.bfloat16)
    tg = torch.randint(0, 10, (2, 50), generator=g).to("cuda")
    tg[:, 40:] = 0
    got = codec_tokens.codec_ce_loss(logits, tg)
    ref = torch.nn.functional.cross_entropy(logits.float().view(-1, 10), tg.view(-1), ignore_index=0)
    assert abs(got.item() - ref.item()) <= 1e-5 * abs(ref.item())
