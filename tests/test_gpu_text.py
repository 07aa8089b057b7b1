"""GPU parity of the text encoder / duration predictor.

* Against the REFERENCE text_encoder.py itself (tests/golden/text.npz, made
  by tests/golden/make_golden.py importing /root/reference/text_encoder.py
  behind a lib.FastSpeech2 shim): TextEncoder.forward in train mode and in
  the eval branch for L > max_seq_len, every parameter gradient, a
  zero-length row; DurationPredictor forward + compute_loss and gradients.
  fp32 HIP path vs the float64 reference, per tensor max|err| <= 1e-4 *
  max|ref| (the north star's fp32 tolerance is 1e-3).  The FastSpeech2
  internals the shim restates (FFTBlock, VariancePredictor, the sinusoid
  table) are third-party, unvendored and unpinned upstream: that restatement
  is parity unpinned; the reference's own code around it is pinned.
* Against the oracle's float64 restatement at a second, wider config."""
import numpy as np
import pytest
import torch

from test_gpu_ops import close, DEV
from oracle import mamba_ref as R

pytestmark = pytest.mark.gpu


def _perturb(m, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn(p.shape, generator=g))
            elif n.endswith("bias"):
                p.copy_(0.1 * torch.randn(p.shape, generator=g))


def _batch(B, L, V, seed):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, V, (B, L), generator=g)
    lens = torch.randint(L // 2, L + 1, (B,), generator=g)
    lens[0] = L
    mask = torch.arange(L)[None] >= lens[:, None]          # True = pad
    ids[mask] = 0
    return ids, mask


@pytest.mark.parametrize("d_model,n_head,d_k,d_inner", [(64, 2, 16, 128), (512, 2, 64, 1024)])
def test_text_encoder_vs_oracle(d_model, n_head, d_k, d_inner):
    import text_encoder as te
    torch.manual_seed(0)
    V, B, L = 40, 3, 37
    m = te.TextEncoder(V, d_model=d_model, n_layers=2, n_head=n_head, d_k=d_k, d_v=d_k, d_inner=d_inner,
                       dropout=0.0, max_seq_len=100)
    _perturb(m, 1)
    m = m.to(DEV).train()
    ids, mask = _batch(B, L, V, 2)
    out = m(ids.to(DEV), mask=mask.to(DEV))
    w = torch.randn(out.shape)
    (out * w.to(DEV)).sum().backward()
    p = {k: v.detach().cpu().double().requires_grad_(v.requires_grad) for k, v in m.state_dict().items()}
    for k, v in m.named_parameters():
        p[k].requires_grad_(True)
    ref = R.text_encoder_ref(p, ids, mask, 2, n_head, d_k)
    close(out, ref.detach(), rtol=1e-4, name="enc_out")
    (ref * w.double()).sum().backward()
    for k, v in m.named_parameters():
        if not v.requires_grad:
            continue
        if p[k].grad.abs().max() < 1e-9:
            # the key bias: softmax is shift-invariant per query row, so its exact
            # gradient is 0; fp32 leaves rounding noise far below the other grads
            assert v.grad.abs().max().item() < 1e-5, k
            continue
        close(v.grad, p[k].grad, rtol=1e-4, name=k)
    # padding row of the phoneme table gets no gradient, the position table none at all
    assert torch.count_nonzero(m.phoneme_emb.weight.grad[0]) == 0
    assert m.position_enc.grad is None
    close(m.position_enc.detach()[0], R.sinusoid_table_ref(101, d_model, 0), rtol=1e-6, name="position_enc")
    for blk in m.layer_stack:   # the k = 9 weights stay [O][K][C] in storage and so do their gradients
        wk = blk.pos_ffn.w_1.weight
        assert wk.permute(0, 2, 1).is_contiguous() and wk.grad.stride() == wk.stride()


def test_duration_predictor_and_loss_vs_oracle():
    import text_encoder as te
    torch.manual_seed(3)
    B, L, d = 3, 29, 64
    dp = te.DurationPredictor(d_model=d, filter_size=128, kernel_size=3, dropout=0.0)
    _perturb(dp, 4)
    dp = dp.to(DEV)
    x = torch.randn(B, L, d)
    _, mask = _batch(B, L, 10, 5)
    xg = x.to(DEV).requires_grad_(True)
    out = dp(xg, mask=mask.to(DEV))
    target = torch.randint(1, 9, (B, L)).float()
    loss = dp.compute_loss(out, target.to(DEV), mask=mask.to(DEV))
    loss.backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in dp.state_dict().items()}
    xr = x.double().requires_grad_(True)
    ref = R.duration_predictor_ref(p, xr, mask)
    lref = torch.nn.functional.mse_loss(ref, torch.log(target.double() + 1e-8), reduction="none")
    lref = lref.masked_fill(mask, 0.0).sum() / (~mask).sum()
    close(out, ref.detach(), rtol=1e-4, name="log_dur")
    close(loss, lref.detach(), rtol=1e-4, name="loss")
    lref.backward()
    close(xg.grad, xr.grad, rtol=1e-4, name="dx")
    for k, v in dp.named_parameters():
        close(v.grad, p[k].grad, rtol=1e-4, name=k)


def _load_sd(mod, g, prefix):
    sd = {k[len(prefix):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(prefix)}
    mod.load_state_dict(sd)


@pytest.mark.parametrize("tag", ["train", "eval"])
def test_text_encoder_vs_reference_golden(golden, tag):
    """TextEncoder (text_encoder.py:87-128) on the HIP path against the
    reference module's own float64 output and gradients: padded rows, the
    padding id inside a valid span (its embedding row gets no gradient), and
    (eval) the fresh unzeroed position table for L > max_seq_len (:107-112)."""
    import text_encoder as te
    g = golden("text.npz")
    m = te.TextEncoder(40, d_model=64, n_layers=2, n_head=2, d_k=32, d_v=32, d_inner=128, kernel_size=(9, 1),
                       dropout=0.0, max_seq_len=48, padding_idx=0)
    _load_sd(m, g, "enc/sd/")
    m = m.to(DEV).train(tag == "train")
    ids = torch.from_numpy(g[f"{tag}/ids"]).to(DEV)
    mask = torch.from_numpy(g[f"{tag}/mask"]).to(DEV)
    out = m(ids, mask=mask)
    close(out, torch.from_numpy(g[f"{tag}/out"]).double(), rtol=1e-4, name=f"{tag}/out")
    (out * torch.from_numpy(g[f"{tag}/w"]).to(DEV)).sum().backward()
    names = [k[len(f"{tag}/grad/"):] for k in g if k.startswith(f"{tag}/grad/")]
    params = dict(m.named_parameters())
    assert set(names) == {k for k, v in params.items() if v.requires_grad}
    for k in names:
        ref = torch.from_numpy(g[f"{tag}/grad/{k}"]).double()
        if ref.abs().max() < 1e-9:
            # the key bias: softmax is shift-invariant per query row (exact 0)
            assert params[k].grad.abs().max().item() < 1e-5, k
            continue
        close(params[k].grad, ref, rtol=1e-4, name=k)
    assert torch.count_nonzero(m.phoneme_emb.weight.grad[0]) == 0


def test_text_encoder_zero_length_row_vs_reference_golden(golden):
    """A zero-length row: every key padded, the attention row is NaN and the
    reference's masked_fill zeroes it (the HIP path's select does the same);
    the other rows match the reference."""
    import text_encoder as te
    g = golden("text.npz")
    m = te.TextEncoder(40, d_model=64, n_layers=2, n_head=2, d_k=32, d_v=32, d_inner=128, dropout=0.0,
                       max_seq_len=48)
    _load_sd(m, g, "enc/sd/")
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(g["empty/ids"]).to(DEV), mask=torch.from_numpy(g["empty/mask"]).to(DEV))
    assert torch.isfinite(out).all() and not out[1].any()
    close(out, torch.from_numpy(g["empty/out"]).double(), rtol=1e-4, name="empty/out")


def test_duration_predictor_vs_reference_golden(golden):
    """DurationPredictor forward, compute_loss (masked; a zero duration inside
    a valid span) and the unmasked mean, and the input / parameter gradients
    of the masked loss, against the reference module (text_encoder.py:131-209)."""
    import text_encoder as te
    g = golden("text.npz")
    dp = te.DurationPredictor(d_model=64, filter_size=128, kernel_size=3, dropout=0.0)
    _load_sd(dp, g, "dur/sd/")
    dp = dp.to(DEV).train()
    x = torch.from_numpy(g["dur/x"]).to(DEV).requires_grad_(True)
    mask = torch.from_numpy(g["dur/mask"]).to(DEV)
    target = torch.from_numpy(g["dur/target"]).to(DEV)
    pred = dp(x, mask=mask)
    close(pred, torch.from_numpy(g["dur/pred"]).double(), rtol=1e-4, name="pred")
    loss = dp.compute_loss(pred, target, mask=mask)
    close(loss.reshape(1), torch.from_numpy(g["dur/loss"]).double().reshape(1), rtol=1e-4, name="loss")
    loss.backward()
    close(x.grad, torch.from_numpy(g["dur/dx"]).double(), rtol=1e-4, name="dx")
    for k, v in dp.named_parameters():
        close(v.grad, torch.from_numpy(g[f"dur/grad/{k}"]).double(), rtol=1e-4, name=k)
    with torch.no_grad():
        nm = dp.compute_loss(dp(x.detach(), mask=None), target.clamp(min=1.0))
    close(nm.reshape(1), torch.from_numpy(g["dur/loss_nomask"]).double().reshape(1), rtol=1e-4, name="loss_nomask")


def test_text_encoder_int32_ids_backward():
    """int32 phoneme ids (F.embedding accepts them) run forward and backward
    and give the int64 ids' gradients."""
    import text_encoder as te
    torch.manual_seed(0)
    m = te.TextEncoder(40, d_model=64, n_layers=1, n_head=2, d_k=32, d_v=32, d_inner=128, dropout=0.0).to(DEV)
    ids, mask = _batch(2, 20, 40, 9)
    grads = []
    for dt in (torch.int64, torch.int32):
        m.zero_grad(set_to_none=True)
        m(ids.to(DEV, dt), mask=mask.to(DEV)).square().sum().backward()
        grads.append(m.phoneme_emb.weight.grad.clone())
    assert torch.equal(grads[0], grads[1])
