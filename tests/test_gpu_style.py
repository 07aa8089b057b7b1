"""GPU parity of the style pipeline's hot spots:
the HIP length regulator (mtts_length_regulate_*) and the single-key
cross-attention path, against the reference's own outputs
(tests/golden/regulator.npz) and the CPU oracle (oracle/mamba_ref.py).
Integer work (lengths, which row lands where) is exact; values are copies
(exact) and the backward sums in fp32 (1e-6 / bf16 1e-2 relative)."""
import numpy as np
import pytest
import torch

from test_gpu_ops import close, DEV
from oracle import mamba_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag,max_len", [("none", None), ("short", 6), ("long", 40)])
def test_regulator_vs_reference_golden(golden, tag, max_len):
    from mtts import ops
    g = golden("regulator.npz")
    h = torch.from_numpy(g["hidden"]).to(DEV).requires_grad_(True)
    out, lengths = ops.length_regulate(h, torch.from_numpy(g["durations"]).to(DEV), max_len)
    assert torch.equal(lengths.cpu(), torch.from_numpy(g[f"{tag}/lengths"]))
    assert out.shape == g[f"{tag}/out"].shape
    assert torch.equal(out.detach().cpu(), torch.from_numpy(g[f"{tag}/out"]))   # rows are copies: exact
    (out * torch.from_numpy(g[f"{tag}/w"]).to(DEV)).sum().backward()
    close(h.grad, g[f"{tag}/dhidden"], rtol=1e-6, name="dhidden")


def _ragged(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    d = torch.randint(0, 7, (B, T), generator=g).float()
    d += torch.randint(0, 2, (B, T), generator=g).float() * 0.5       # .5 ties (half to even)
    d[torch.rand(B, T, generator=g) < 0.1] = -1.5                     # clamp
    if B > 1:
        d[1] = 0.0                                                    # an empty row
    return d


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T,D,pad", [(3, 17, 64, 0), (2, 5, 20, 0), (2, 33, 24, 8), (1, 1, 8, 0),
                                       (2, 300, 512, 0), (2, 4096, 16, 0)])
@pytest.mark.parametrize("max_len", [None, 9, 5000])
def test_regulator_vs_oracle(dtype, B, T, D, pad, max_len):
    """Ragged durations, vector (16-byte rows) and element paths (D=20 bf16),
    strided hidden (pad > 0: a column slice of a wider tensor), T at the
    4096 maximum, max_len None / truncating / padding; grads through the
    segment-sum backward."""
    from mtts import ops
    torch.manual_seed(0)
    dur = _ragged(B, T, seed=B * 1000 + T)
    full = torch.randn(B, T, D + pad).to(dtype)
    h_cpu = full[..., :D]
    h = full.to(DEV)[..., :D].detach().requires_grad_(True)
    out, lengths = ops.length_regulate(h, dur.to(DEV), max_len)
    ref, ref_len = R.length_regulator_ref(h_cpu.double(), dur.double(), max_len)
    assert torch.equal(lengths.cpu(), ref_len)
    assert out.shape == ref.shape
    assert torch.equal(out.detach().cpu().double(), ref)
    w = torch.randn(out.shape)
    (out * w.to(DEV, dtype)).sum().backward()
    hr = h_cpu.double().requires_grad_(True)
    o2, _ = R.length_regulator_ref(hr, dur.double(), max_len)
    (o2 * w.to(dtype).double()).sum().backward()
    close(h.grad, hr.grad.numpy(), rtol=1e-6 if dtype == torch.float32 else 1e-2, name="dhidden")


def test_regulator_limits():
    from mtts import ops
    h = torch.randn(1, 4097, 8, device=DEV)
    with pytest.raises(RuntimeError, match="4096"):
        ops.length_regulate(h, torch.ones(1, 4097, device=DEV))
    out, lengths = ops.length_regulate(torch.randn(2, 3, 8, device=DEV), torch.zeros(2, 3, device=DEV))
    assert out.shape == (2, 0, 8) and lengths.tolist() == [0, 0]


@pytest.mark.parametrize("Tq", [1, 37, 300])
def test_single_key_attention_vs_oracle(Tq):
    """CrossAttention with one unmasked key (the style token): out_proj(v)
    shortcut vs the oracle's full MHA, outputs and every gradient (q/k rows of
    the in-projection get exactly zero, as in torch MHA; `key` gets a zero
    gradient, not None)."""
    from mtts.attention import CrossAttention
    torch.manual_seed(1)
    d, H, B = 64, 4, 3
    m = CrossAttention(d, H, dropout=0.0).to(DEV)
    with torch.no_grad():
        m.in_proj_bias.normal_()
        m.out_proj.bias.normal_()
    q = torch.randn(B, Tq, d, device=DEV, requires_grad=True)
    k = torch.randn(B, 1, d, device=DEV, requires_grad=True)
    v = torch.randn(B, 1, d, device=DEV, requires_grad=True)
    out, _ = m(q, k, v)
    w = torch.randn_like(out)
    (out * w).sum().backward()
    P = {n: t.detach().cpu().double().requires_grad_(True) for n, t in
         [("in_w", m.in_proj_weight), ("in_b", m.in_proj_bias), ("out_w", m.out_proj.weight),
          ("out_b", m.out_proj.bias), ("q", q), ("k", k), ("v", v)]}
    # the oracle MHA takes one kv input: feed k for the key rows and v for the value rows
    qd, kd, vd = P["q"], P["k"], P["v"]
    qq = qd @ P["in_w"][:d].T + P["in_b"][:d]
    kk = kd @ P["in_w"][d:2 * d].T + P["in_b"][d:2 * d]
    vv = vd @ P["in_w"][2 * d:].T + P["in_b"][2 * d:]
    hd = d // H
    s = (qq.view(B, Tq, H, hd).transpose(1, 2) @ kk.view(B, 1, H, hd).transpose(1, 2).transpose(-1, -2)) / hd ** 0.5
    o = (torch.softmax(s, -1) @ vv.view(B, 1, H, hd).transpose(1, 2)).transpose(1, 2).reshape(B, Tq, d)
    ref = o @ P["out_w"].T + P["out_b"]
    close(out, ref.detach().numpy(), name="out")
    (ref * w.cpu().double()).sum().backward()
    for name, t in [("in_w", m.in_proj_weight.grad), ("in_b", m.in_proj_bias.grad), ("out_w", m.out_proj.weight.grad),
                    ("out_b", m.out_proj.bias.grad), ("v", v.grad)]:
        close(t, P[name].grad.numpy(), name=name)
    assert k.grad is not None and torch.count_nonzero(k.grad) == 0
    assert q.grad is None or torch.count_nonzero(q.grad) == 0
    assert torch.count_nonzero(m.in_proj_weight.grad[:2 * d]) == 0
