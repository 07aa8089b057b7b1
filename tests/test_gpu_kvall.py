"""All decoder layers' cross-attention K/V projections as ONE GEMM
(mtts.attention.KVAllFn, used by MambaTTSDecoder._run_layers): the same
forward and gradients as the per-layer projections (reference
mamba_decoder.py:72-77, nn.MultiheadAttention's packed in_proj per layer),
with the attention backward writing every layer's dK / dV into one sink and
the key gradient summed over layers inside one GEMM."""
import pytest
import torch

from test_gpu_ops import close, DEV

pytestmark = pytest.mark.gpu


def _run(model, batch, batched, deferred, monkeypatch):
    import mamba_decoder
    from mtts import wgrad
    from mtts.attention import kv_all_ok
    monkeypatch.setattr(mamba_decoder, "kv_all_ok", kv_all_ok if batched else (lambda k, a: False))
    tokens, text, z, mask = batch
    for p in model.parameters():
        p.grad = None
    th = text.detach().clone().requires_grad_(True)
    out = model(tokens, th, z, text_mask=mask)
    g = torch.Generator(device=DEV).manual_seed(9)
    gy = torch.randn(out.shape, device=DEV, generator=g).to(out.dtype)
    with wgrad.deferred(deferred):
        out.backward(gy)
    return out.detach(), th.grad.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()
                                             if p.grad is not None}


@pytest.mark.parametrize("cd,deferred", [(torch.float32, False), (torch.bfloat16, False), (torch.bfloat16, True)])
def test_decoder_kv_all_equals_per_layer_projections(cd, deferred, monkeypatch):
    import mamba_decoder
    from mtts import attention as A
    torch.manual_seed(0)
    d, B, T, Tt = 256, 2, 192, 96
    model = mamba_decoder.MambaTTSDecoder(12, d_model=d, n_layers=3, n_heads=4, d_ff=512, d_style=64).to(DEV)
    model.compute_dtype = cd
    tokens = torch.randint(0, 12, (B, T), device=DEV)
    text = torch.randn(B, Tt, d, device=DEV)
    z = torch.randn(B, 64, device=DEV)
    mask = torch.ones(B, Tt, dtype=torch.bool, device=DEV)
    mask[1, 70:] = False
    calls = []
    orig = A.KVAllFn.backward

    def spy(ctx, *dkvs):
        calls.append(ctx.sink.buf is not None)
        return orig(ctx, *dkvs)
    monkeypatch.setattr(A.KVAllFn, "backward", staticmethod(spy))
    ref = _run(model, (tokens, text, z, mask), False, deferred, monkeypatch)
    assert not calls
    new = _run(model, (tokens, text, z, mask), True, deferred, monkeypatch)
    assert calls == [True]          # the batched path ran, every layer's dK / dV landed in the sink
    tol = 1e-4 if cd == torch.float32 else 3e-2
    close(new[0].float(), ref[0].float(), rtol=tol, name="logits")
    close(new[1].float(), ref[1].float(), rtol=tol, name="d text_hidden")
    assert set(new[2]) == set(ref[2])
    for n in ref[2]:
        close(new[2][n], ref[2][n], rtol=tol, name=n)


def test_kv_all_backward_twice_through_a_retained_graph():
    """retain_graph: a second backward through the same forward (the K/V sink
    re-armed) adds exactly the first backward's gradients again."""
    import mamba_decoder
    torch.manual_seed(1)
    d, B, T, Tt = 256, 2, 128, 64
    model = mamba_decoder.MambaTTSDecoder(12, d_model=d, n_layers=2, n_heads=4, d_ff=512, d_style=64).to(DEV)
    model.compute_dtype = torch.bfloat16
    tokens = torch.randint(0, 12, (B, T), device=DEV)
    text = torch.randn(B, Tt, d, device=DEV, requires_grad=True)
    z = torch.randn(B, 64, device=DEV)
    out = model(tokens, text, z)
    gy = torch.randn(out.shape, device=DEV).to(out.dtype)
    out.backward(gy, retain_graph=True)
    once = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    t1 = text.grad.clone()
    out.backward(gy)
    for n, p in model.named_parameters():
        if n in once:
            close(p.grad, 2 * once[n], rtol=1e-5, name=n)
    close(text.grad, 2 * t1, rtol=1e-2, name="d text_hidden")
