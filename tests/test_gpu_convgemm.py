"""fp32 windowed-row MFMA GEMM (csrc/convgemm.hip, mtts.convgemm) against
torch fp32: plain NT / TN / NN products (one workgroup per tile and split-K) with
ragged edges and every epilogue,
'same' convolutions (k = 9 / 3 / 1) forward and backward against
F.conv1d's autograd, the fused conv FFN against its unfused composition, and
the argument checks.  The text encoder's / duration predictor's
convolutions (reference text_encoder.py:80-85, 118-122, 131-209 via
FastSpeech2's Conv1d) run on these.

Tolerance: exact-f32 MFMA products with fp32 accumulation in a different
order than torch's: 1e-5 of each tensor's max |value|."""
import pytest
import torch
import torch.nn.functional as F

from mtts import convgemm as CG

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(x, ref):
    return ((x - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("m,n,k", [(64, 64, 32), (1000, 388, 516), (7, 4, 4), (1024, 1536, 512), (130, 260, 36)])
def test_nt_tn_plain_and_epilogues(m, n, k):
    torch.manual_seed(m + n + k)
    a, b = torch.randn(m, k, device=dev), torch.randn(n, k, device=dev)
    bias = torch.randn(n, device=dev)
    ref = a @ b.t()
    c = torch.empty(m, n, device=dev)
    CG.gemm(CG.NT, m, n, k, CG._plain(a), CG._plain(b), CG._plain(c))
    assert rel(c, ref) < 1e-5
    CG.gemm(CG.NT, m, n, k, CG._plain(a), CG._plain(b), CG._plain(c), bias=bias, epilogue=CG.EPI_BIAS | CG.EPI_RELU)
    assert rel(c, torch.relu(ref + bias)) < 1e-5
    aux = torch.randn(m, n, device=dev)
    CG.gemm(CG.NT, m, n, k, CG._plain(a), CG._plain(b), CG._plain(c), epilogue=CG.EPI_DRELU, aux=CG._plain(aux))
    assert rel(c, torch.where(aux > 0, ref, torch.zeros(()).to(dev))) < 1e-5
    before = torch.randn(m, n, device=dev)
    c.copy_(before)
    CG.gemm(CG.NT, m, n, k, CG._plain(a), CG._plain(b), CG._plain(c), beta=1.0)
    assert rel(c, ref + before) < 1e-5
    bkn = torch.randn(k, n, device=dev)   # NN: C = A B with B row-major (k, n)
    CG.gemm(CG.NN, m, n, k, CG._plain(a), CG._plain(bkn), CG._plain(c))
    assert rel(c, a @ bkn) < 1e-5
    if m % 4 == 0:   # TN: C = A^T B over row-major (k, m) / (k, n)
        at, bt = torch.randn(k, m, device=dev), torch.randn(k, n, device=dev)
        CG.gemm(CG.TN, m, n, k, CG._plain(at), CG._plain(bt), CG._plain(c))
        assert rel(c, at.t() @ bt) < 1e-5
        # the column sums of A (the bias gradient when A = dy) from the same launch(es)
        cs = torch.full((m,), float("nan"), device=dev)
        c.zero_()
        CG.gemm(CG.TN, m, n, k, CG._plain(at), CG._plain(bt), CG._plain(c), colsum_a=cs)
        assert rel(c, at.t() @ bt) < 1e-5 and rel(cs, at.sum(0)) < 1e-5


@pytest.mark.parametrize("B,T,C,O,K", [(8, 128, 512, 1024, 9), (2, 13, 64, 128, 9), (3, 40, 256, 256, 3),
                                       (2, 9, 64, 64, 1), (1, 5, 32, 36, 3)])
@pytest.mark.parametrize("relu", [False, True])
def test_conv1d_same_fwd_bwd_vs_torch(B, T, C, O, K, relu):
    """Channel-last 'same' Conv1d (padding (K-1)/2) vs F.conv1d: output, dx,
    dW, db; the first and last K/2 steps read the zero padding."""
    torch.manual_seed(B * T + K)
    x = torch.randn(B, T, C, device=dev, requires_grad=True)
    w = (torch.randn(O, C, K, device=dev) / (C * K) ** 0.5).requires_grad_(True)
    b = torch.randn(O, device=dev, requires_grad=True)
    g = torch.randn(B, T, O, device=dev)
    y = CG.conv1d_same(x, w, b, relu=relu)
    (y * g).sum().backward()
    got = [y.detach(), x.grad, w.grad, b.grad]
    x2, w2, b2 = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv1d(x2.transpose(1, 2), w2, b2, padding=(K - 1) // 2).transpose(1, 2)
    if relu:
        assert rel(got[0], torch.relu(yr.detach())) < 1e-5, "y"
        # the backward on the kernel's own ReLU mask: a pre-activation within
        # fp32 rounding of 0 may take the other side of the kink in torch
        yr = yr * (got[0] > 0)
    (yr * g).sum().backward()
    for name, a, r in zip(("y", "dx", "dW", "db"), got, [yr.detach(), x2.grad, w2.grad, b2.grad]):
        assert rel(a, r) < 1e-5, name


def test_conv_ffn_matches_composition():
    """ConvFFNFn (ReLU fused into conv 1's epilogue, its backward into conv 2's
    data-gradient epilogue) vs two Conv1dFn calls."""
    torch.manual_seed(3)
    B, T, C, H = 4, 50, 128, 256
    x = torch.randn(B, T, C, device=dev)
    w1, b1 = torch.randn(H, C, 9, device=dev) / 34, torch.randn(H, device=dev)
    w2, b2 = torch.randn(C, H, 1, device=dev) / 16, torch.randn(C, device=dev)
    g = torch.randn(B, T, C, device=dev)
    outs = []
    for fused in (True, False):
        ts = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
        if fused:
            y = CG.conv_ffn(*ts)
        else:
            y = CG.conv1d_same(CG.conv1d_same(ts[0], ts[1], ts[2], relu=True), ts[3], ts[4])
        (y * g).sum().backward()
        outs.append([y.detach()] + [t.grad for t in ts])
    for a, r in zip(*outs):
        assert rel(a, r) < 1e-6


def test_linear_narrow_output_and_3d():
    torch.manual_seed(4)
    x = torch.randn(3, 17, 64, device=dev, requires_grad=True)
    w = torch.randn(1, 64, device=dev, requires_grad=True)
    b = torch.randn(1, device=dev, requires_grad=True)
    y = CG.linear(x, w, b)
    y.square().sum().backward()
    x2, w2, b2 = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = F.linear(x2, w2, b2)
    yr.square().sum().backward()
    for a, r in ((y, yr), (x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        assert a.shape == r.shape and rel(a.detach(), r.detach()) < 1e-5


def test_refuses_bad_arguments():
    a = torch.randn(8, 8, device=dev)
    c = torch.empty(8, 8, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 4"):
        CG.gemm(CG.NT, 8, 6, 8, CG._plain(a), CG._plain(a), CG._plain(c))
    with pytest.raises(RuntimeError, match="bias"):
        CG.gemm(CG.NT, 8, 8, 8, CG._plain(a), CG._plain(a), CG._plain(c), epilogue=CG.EPI_BIAS)
    with pytest.raises(RuntimeError, match="colsum_a"):
        CG.gemm(CG.NT, 8, 8, 8, CG._plain(a), CG._plain(a), CG._plain(c), colsum_a=torch.empty(8, device=dev))
    with pytest.raises(TypeError):
        CG.conv1d_same(torch.randn(1, 4, 8, device=dev, dtype=torch.bfloat16), torch.randn(8, 8, 3, device=dev))


@pytest.mark.parametrize("B,T,C,K", [(3, 40, 64, 9), (2, 3, 32, 9), (4, 17, 96, 3)])
def test_halo_windows_equal_padded_copy(B, T, C, K, monkeypatch):
    """The halo row map (taps outside [0, T) read as zeros in the kernel) gives
    bit-identical forward / dx / dW to the explicitly zero-padded windows,
    including T < p (every tap of a row but a few reads the halo)."""
    torch.manual_seed(B * T * K)
    x = torch.randn(B, T, C, device=dev)
    w = torch.randn(64, C, K, device=dev) / (C * K) ** 0.5
    b = torch.randn(64, device=dev)
    g = torch.randn(B, T, 64, device=dev)
    outs = []
    for halo in (True, False):
        if not halo:
            monkeypatch.setattr(CG, "_halo_ok", lambda C_, p: False)
        ts = [t.clone().requires_grad_(True) for t in (x, w, b)]
        y = CG.conv1d_same(*ts)
        (y * g).sum().backward()
        outs.append([y.detach()] + [t.grad for t in ts])
    for a, r in zip(*outs):
        assert torch.equal(a, r)
