"""GPU parity of the text encoder / duration predictor
against the oracle's float64 restatement of FastSpeech2's FFTBlock /
VariancePredictor (oracle.text_encoder_ref, duration_predictor_ref).
PARITY UNPINNED: the reference builds these from ming024/FastSpeech2, which
it neither vendors nor pins and which is absent here, so no reference output
exists to pin the restatement to.  fp32, 1e-4 relative;
dropout off (eval) for values, train-mode gradients with dropout 0."""
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
