"""Host-side pieces of the training step on CPU: the fused embedding-sum
backward (mtts/embed.py) against nn.Embedding autograd, and clip-in-optimizer
(mtts/optim.py) against clip_grad_norm_ + the same optimizer."""
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("vocab", [10, 300])
def test_embed_sum_matches_nn_embedding(vocab):
    from mtts.embed import embed_sum
    g = torch.Generator().manual_seed(0)
    B, T, d, Q, P = 3, 17, 8, 4, 32
    tok = torch.randint(0, vocab, (B, T), generator=g)
    qid = torch.randint(0, Q, (B, T), generator=g)
    tw = torch.randn(vocab, d, generator=g, requires_grad=True)
    qw = torch.randn(Q, d, generator=g, requires_grad=True)
    pw = torch.randn(P, d, generator=g, requires_grad=True)
    dy = torch.randn(B, T, d, generator=g)
    x = embed_sum(tok, qid, tw, qw, pw, torch.float32)
    x.backward(dy)
    got = [t.grad.clone() for t in (tw, qw, pw)]
    for t in (tw, qw, pw):
        t.grad = None
    ref = F.embedding(tok, tw) + F.embedding(qid, qw) + F.embedding(torch.arange(T), pw)[None]
    torch.testing.assert_close(x, ref)
    ref.backward(dy)
    for a, t in zip(got, (tw, qw, pw)):
        torch.testing.assert_close(a, t.grad, rtol=1e-5, atol=1e-5)


def test_clip_into_optimizer_equals_clip_grad_norm():
    from mtts.optim import clip_into_optimizer
    torch.manual_seed(0)
    try:
        torch.optim.Adam([torch.zeros(1, requires_grad=True)], fused=True)
    except Exception as e:  # pragma: no cover
        pytest.skip(f"fused Adam unavailable on CPU: {e}")
    ps1 = [torch.randn(7, 5, requires_grad=True), torch.randn(11, requires_grad=True)]
    ps2 = [p.detach().clone().requires_grad_(True) for p in ps1]
    o1 = torch.optim.Adam(ps1, lr=1e-2, fused=True)
    o2 = torch.optim.Adam(ps2, lr=1e-2, fused=True)
    for step in range(3):
        gs = [torch.randn_like(p) * 10 for p in ps1]
        for p, gg in zip(ps1, gs):
            p.grad = gg.clone()
        for p, gg in zip(ps2, gs):
            p.grad = gg.clone()
        n1 = torch.nn.utils.clip_grad_norm_(ps1, 1.0)
        o1.step()
        n2 = clip_into_optimizer(o2, ps2, 1.0)
        o2.step()
        torch.testing.assert_close(n1, n2)
        for a, b in zip(ps1, ps2):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
