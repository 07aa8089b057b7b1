"""HIP dropout (csrc/dropout.hip, mtts/dropout.py) and the paths built on it:
the style blocks' FFN with dropout between GELU and the second linear
(mtts.linear.FFNFn, p > 0), the single-key attention with attention-weight
dropout (mtts.attention.CrossAttention._single_key), and the text encoder /
style pipeline in training mode.  Dropout draws cannot match torch's element
for element, so the tests check the mask's statistics, that the backward
regenerates the forward's mask, and the arithmetic around the mask against a
float64 torch reference that uses the SAME mask (read back from the kernel
by dropping a tensor of ones with the same seed)."""
import math

import pytest
import torch

from test_gpu_ops import close, DEV

pytestmark = pytest.mark.gpu


def _mask(shape, p, seed, group=1, dtype=torch.float32):
    from mtts import dropout as DO
    ones = torch.ones(shape, device=DEV, dtype=dtype)
    return DO.apply_mask(ones, p, seed, group=group) * (1.0 - p)    # 0 / 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_dropout_kernel_statistics_and_values(dtype, p):
    from mtts import dropout as DO
    n = 1 << 23
    x = torch.randn(n, device=DEV).to(dtype)
    y = DO.apply_mask(x, p, seed=12345)
    keep = y != 0
    frac = keep.float().mean().item()
    sd = math.sqrt(p * (1 - p) / n)
    assert abs(frac - (1 - p)) < 6 * sd, frac
    # survivors are x / (1 - p) rounded once to the I/O dtype
    exp = (x.float() / (1 - p)).to(dtype)
    assert torch.equal(y[keep], exp[keep])
    assert torch.equal(y[~keep], torch.zeros_like(y[~keep]))
    # the same seed gives the same mask; another seed an independent one
    assert torch.equal(DO.apply_mask(x, p, seed=12345), y)
    keep2 = DO.apply_mask(x, p, seed=777) != 0
    both = (keep & keep2).float().mean().item()
    assert abs(both - (1 - p) ** 2) < 6 * sd
    # neighbouring elements are independent (the pair hash's two halves)
    adj = (keep[0::2] & keep[1::2]).float().mean().item()
    assert abs(adj - (1 - p) ** 2) < 8 * math.sqrt(p * (1 - p) / (n // 2))


def test_dropout_group_one_draw_per_group():
    from mtts import dropout as DO
    B, T, H, hd = 4, 300, 8, 64
    m = _mask((B, T, H * hd), 0.3, seed=99, group=hd, dtype=torch.bfloat16).view(B, T, H, hd)
    assert torch.equal(m.amax(-1), m.amin(-1))            # constant within a head's slice
    frac = m[..., 0].float().mean().item()
    assert abs(frac - 0.7) < 0.02
    with pytest.raises(RuntimeError):
        DO.apply_mask(torch.ones(64, device=DEV), 0.1, 1, group=6)


@pytest.mark.parametrize("dtype,R", [(torch.float32, 37), (torch.bfloat16, 37), (torch.bfloat16, 1090)])
def test_dropout_broadcast_source_equals_the_expanded_copy(dtype, R):
    """rep > 1 (ABI 14): x (O, C) read as x[o] for every y[o, r] -- the same
    output, bit for bit, as dropping the materialised expand; the autograd form's
    backward sums the masked gradient over each o's rows (fp32)."""
    from mtts import dropout as DO
    O, Cn, p, seed = 3, 256, 0.25, 777     # R = 1090: the column sums' ragged > 1024-row groups
    x = torch.randn(O, Cn, device=DEV).to(dtype)
    for group in (1, 64):
        y = DO.apply_mask(x, p, seed, group=group, rep=R)
        ref = DO.apply_mask(x[:, None, :].expand(O, R, Cn).contiguous(), p, seed, group=group)
        assert y.shape == (O, R, Cn) and torch.equal(y, ref)
    with pytest.raises(RuntimeError):
        DO.apply_mask(torch.randn(4, 6, device=DEV), p, seed, rep=R)      # rows of 6 fp32: not whole 16-byte pieces
    xg = x.float().requires_grad_(True)
    torch.manual_seed(3)
    y = DO.dropout_bcast(xg, R, p, group=64)
    g = torch.randn_like(y)
    y.backward(g)
    keep = (y != 0).float() / (1 - p)
    close(xg.grad, (g.double() * keep).sum(1), rtol=1e-5, name="dx")


def test_dropout_fn_backward_regenerates_the_mask():
    from mtts import dropout as DO
    torch.manual_seed(0)
    x = torch.randn(1000, 24, device=DEV, requires_grad=True)
    y = DO.dropout(x, 0.2, True)
    g = torch.randn_like(y)
    y.backward(g)
    keep = (y != 0).float()
    close(x.grad, g * keep / 0.8, rtol=1e-6, name="dx")
    assert DO.dropout(x, 0.2, False) is x and DO.dropout(x, 0.0, True) is x
    # odd sizes (numel % 8 != 0) are padded to the kernel's granule
    z = torch.randn(3, 5, device=DEV, requires_grad=True)
    DO.dropout(z, 0.5, True).sum().backward()
    assert z.grad.shape == z.shape


def test_dropout_in_a_replayed_graph_draws_fresh_masks():
    """A training step captured in a hipGraph (CPU seeds frozen at capture)
    draws a new mask on every replay when it advances the device seed base
    (mtts.dropout.advance, captured); the backward of each replay uses its
    own forward's mask (the base recorded per call), also when the base moves
    between a forward and its backward (eager)."""
    from mtts import dropout as DO
    base = DO.device_base(DEV)
    try:
        torch.manual_seed(0)
        x = torch.randn(4096, 64, device=DEV, requires_grad=True)
        g = torch.randn(4096, 64, device=DEV)
        static = {}

        def step():
            DO.advance()
            x.grad = None
            y = DO.dropout(x, 0.3, True)
            y.backward(g)
            static["y"], static["dx"] = y.detach(), x.grad

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        masks = []
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            keep = static["y"] != 0
            masks.append(keep.clone())
            close(static["dx"], g * keep / 0.7, rtol=1e-6, name="dx of the same replay")
        assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
        # eager: the base moves between forward and backward -- the backward keeps the forward's mask
        x.grad = None
        y = DO.dropout(x, 0.3, True)
        DO.advance()
        y.backward(g)
        close(x.grad, g * (y != 0) / 0.7, rtol=1e-6, name="dx after advance")
    finally:
        base.zero_()


def test_dropout_dgelu_form():
    """dropout(gelu(pre)) backward in one pass: bf16(bf16(dy * keep / (1 - p)) * gelu'(pre))."""
    from mtts import dropout as DO
    g = torch.Generator(device="cpu").manual_seed(1)
    pre = (torch.randn(4096, 64, generator=g) * 2).to(DEV, torch.bfloat16)
    dy = torch.randn(4096, 64, generator=g).to(DEV, torch.bfloat16)
    p, seed = 0.1, 4242
    out = DO.apply_mask(dy, p, seed, pre=pre)
    m = _mask(dy.shape, p, seed)
    xp = pre.double().requires_grad_(True)
    torch.nn.functional.gelu(xp).backward(torch.ones_like(xp))
    ref = ((dy.float() * m / (1 - p)).to(torch.bfloat16).double() * xp.grad)
    close(out, ref, rtol=1e-2, name="dpre")          # one bf16 rounding of the product
    assert torch.equal(out == 0, m == 0) or bool(((out == 0) | (m != 0)).all())


def test_ffn_with_dropout_matches_reference_with_the_same_mask(monkeypatch):
    """FFNFn(p > 0): gelu(h W1^T + b1) -> dropout -> W2^T + b2, bf16 on the NT
    GEMM, forward and every gradient vs float64 torch with the kernel's mask."""
    from mtts import dropout as DO
    from mtts.linear import ffn
    monkeypatch.setattr(DO, "new_seed", lambda: 2024)
    g = torch.Generator(device="cpu").manual_seed(5)
    M, d, dff, p = 1000, 256, 1024, 0.1
    h = torch.randn(M, d, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    w1 = (torch.randn(dff, d, generator=g) * d ** -0.5).to(DEV).requires_grad_(True)
    b1 = (torch.randn(dff, generator=g) * 0.1).to(DEV).requires_grad_(True)
    w2 = (torch.randn(d, dff, generator=g) * dff ** -0.5).to(DEV).requires_grad_(True)
    b2 = (torch.randn(d, generator=g) * 0.1).to(DEV).requires_grad_(True)
    y = ffn(h, w1, b1, w2, b2, p=p)
    dy = torch.randn(M, d, generator=g).to(DEV, torch.bfloat16)
    y.backward(dy)
    m = _mask((M, dff), p, 2024).double()
    ref_in = [t.detach().double().requires_grad_(True) for t in (h, w1, b1, w2, b2)]
    hh, W1, B1, W2, B2 = ref_in
    a = torch.nn.functional.gelu(hh @ W1.T + B1) * m / (1 - p)
    yr = a @ W2.T + B2
    yr.backward(dy.double())
    close(y, yr, rtol=2e-2, name="y")
    for t, r, nm in zip((h, w1, b1, w2, b2), ref_in, ("dh", "dw1", "db1", "dw2", "db2")):
        close(t.grad, r.grad, rtol=3e-2, name=nm)


def test_single_key_attention_dropout_matches_reference_with_the_same_mask(monkeypatch):
    """nn.MultiheadAttention over ONE key with attention-weight dropout: each
    (batch, query, head) weight 1 kept with probability 1 - p (one HIP draw per
    head slice) -> out_proj; vs float64 with the kernel's mask, fp32."""
    from mtts import dropout as DO
    from mtts.attention import CrossAttention
    monkeypatch.setattr(DO, "new_seed", lambda: 31337)
    torch.manual_seed(0)
    B, T, d, H, p = 3, 40, 128, 4, 0.25
    att = CrossAttention(d, H, dropout=p).to(DEV).train()
    q = torch.randn(B, T, d, device=DEV, requires_grad=True)
    kv = torch.randn(B, 1, d, device=DEV, requires_grad=True)
    o, _ = att(q, kv, kv)
    w = torch.randn_like(o)
    (o * w).sum().backward()
    m = _mask((B, T, d), p, 31337, group=d // H).double()
    W = att.in_proj_weight.detach().double()
    bb = att.in_proj_bias.detach().double()
    v = kv.detach().double() @ W[2 * d:].T + bb[2 * d:]
    o_ref = (v.expand(B, T, d) * m / (1 - p)) @ att.out_proj.weight.detach().double().T + \
        att.out_proj.bias.detach().double()
    close(o, o_ref, rtol=1e-5, name="o")
    frac = m.view(B, T, H, -1)[..., 0].mean().item()
    assert abs(frac - (1 - p)) < 0.1
    assert att.in_proj_weight.grad[:2 * d].abs().max() == 0   # q / k rows: exactly zero, as torch MHA
    assert q.grad is None or q.grad.abs().max() == 0


def test_style_pipeline_and_text_encoder_train_with_hip_dropout():
    """Training-mode forward + backward of the style pipeline (bf16 compute,
    dropout 0.1 everywhere) and of the text encoder (fp32): finite, dropout
    active (two calls differ), every parameter receives a gradient, and no
    F.dropout / torch fused-dropout kernel is needed (the modules call the
    HIP kernel)."""
    import style_cross_attention as sca
    import text_encoder as te
    torch.manual_seed(0)
    pipe = sca.StyleConditioningPipeline(d_style=64, d_model=256, num_heads=4, dropout=0.1).to(DEV).train()
    pipe.compute_dtype = torch.bfloat16
    text = torch.randn(2, 16, 256, device=DEV, requires_grad=True)
    style = torch.randn(2, 64, device=DEV)
    dur = torch.randint(1, 6, (2, 16), device=DEV).float()
    f1, _, _, _ = pipe(text, style, dur)
    f1.float().square().mean().backward()
    with torch.no_grad():   # (the cached bf16 weight copies a graph saved are re-cast by the next forward)
        f2, _, _, _ = pipe(text, style, dur)
    assert f1.dtype == torch.bfloat16 and not torch.equal(f1, f2)
    for n, prm in pipe.named_parameters():
        assert prm.grad is not None and torch.isfinite(prm.grad).all(), n
    enc = te.TextEncoder(20, d_model=64, n_layers=2, n_head=2, d_k=32, d_v=32, d_inner=128, dropout=0.1).to(DEV).train()
    ids = torch.randint(1, 20, (2, 24), device=DEV)
    mask = torch.zeros(2, 24, dtype=torch.bool, device=DEV)
    mask[1, 20:] = True
    o1, o2 = enc(ids, mask=mask), enc(ids, mask=mask)
    assert not torch.equal(o1, o2) and torch.isfinite(o1).all()
    o1.square().mean().backward()
    for n, prm in enc.named_parameters():
        if prm.requires_grad:
            assert prm.grad is not None and torch.isfinite(prm.grad).all(), n
