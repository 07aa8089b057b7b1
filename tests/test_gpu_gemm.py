"""Hand-written MFMA GEMM (csrc/gemm.hip, mtts_gemm) against fp32 products of
the same bf16 operands: NT (forward / data gradient) with bias, GELU and
GELU-backward epilogues, TN (weight gradient) with split-K and accumulate,
ragged and strided shapes, and the fused FFN autograd function against the
per-op path (reference mamba_decoder.py:39-43, 88).

Tolerances: bf16 outputs are checked to 1e-2 of the reference's max (bf16
rounding is 2^-9 relative); fp32 outputs (weight gradients) to 1e-5 of max."""
import pytest
import torch
import torch.nn.functional as F

from mtts import gemm as G
from mtts import linear as LIN

pytestmark = pytest.mark.gpu
dev = "cuda"


def rnd(*s, scale=1.0, dtype=torch.bfloat16):
    return ((torch.rand(*s, device=dev) * 2 - 1) * scale).to(dtype)


def rel(x, ref):
    return ((x.float() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-30)).item()


def gelu_matches(act, pre):
    """The epilogue's GELU of the bf16 pre-activation vs F.gelu of the same
    bf16 values: within one bf16 ulp element-wise (the epilogue evaluates
    erfc through one polynomial + exp2 with <= 2.8e-6 relative error in fp32,
    csrc/gemm.hip gelu_f, so a value next to a rounding boundary may round the
    other way), tiny tail values (|gelu| < 1e-6) within 1e-6 absolute."""
    ref = F.gelu(pre.float())
    return bool(((act.float() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-6).all())


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 128), (1000, 264, 192), (300, 1032, 1024),
                                   (16384, 1024, 1024), (1024, 2048, 1024), (37, 8, 64), (4096, 96, 2048)])
def test_nt_plain(m, n, k):
    torch.manual_seed(m + n + k)
    a, b = rnd(m, k), rnd(n, k)
    out = G.mm_nt(a, b)
    assert rel(out, a.float() @ b.float().t()) < 1e-2


def test_nt_strided_operands_and_output():
    torch.manual_seed(1)
    big_a, big_b = rnd(700, 640), rnd(520, 384)
    a, b = big_a[:, 64:64 + 256], big_b[8:8 + 264, 128:128 + 256]   # row strides 640 / 384
    out_full = torch.zeros(700, 300, device=dev, dtype=torch.bfloat16)
    out = out_full[:, 8:8 + 264]
    G.mm_nt(a, b, out=out)
    assert rel(out, a.float() @ b.float().t()) < 1e-2
    assert out_full[:, :8].abs().max() == 0 and out_full[:, 272:].abs().max() == 0


@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_nt_bias(bias_dtype):
    torch.manual_seed(2)
    a, b, bias = rnd(640, 512), rnd(1024, 512), rnd(1024, dtype=bias_dtype)
    out = G.mm_nt(a, b, bias=bias)
    assert rel(out, a.float() @ b.float().t() + bias.float()) < 1e-2


def test_nt_gelu_epilogue_matches_torch_exactly():
    torch.manual_seed(3)
    a, b, bias = rnd(2048, 1024), rnd(2048, 1024), rnd(2048)
    pre = torch.empty(2048, 2048, device=dev, dtype=torch.bfloat16)
    act = G.mm_nt(a, b, bias=bias, gelu_aux=pre)
    ref_pre = torch.addmm(bias, a, b.t())
    assert rel(pre, ref_pre) < 1e-2
    # the activation is F.gelu of the bf16 pre-activation the kernel wrote
    assert gelu_matches(act, pre)


def test_nt_dgelu_epilogue():
    torch.manual_seed(4)
    dy, w2t, pre = rnd(1536, 1024), rnd(2048, 1024), rnd(1536, 2048, scale=3.0)
    g = G.mm_nt(dy, w2t, dgelu_aux=pre)
    prod = (dy.float() @ w2t.float().t()).to(torch.bfloat16)
    ref = torch.ops.aten.gelu_backward(prod, pre)
    assert rel(g, ref) < 1e-2


@pytest.mark.parametrize("m,n,k,splits", [(1024, 1024, 16384, 8), (4096, 1024, 16384, 4), (264, 520, 2048, 1),
                                          (264, 520, 2048, 2), (96, 2048, 4096, 16), (2048, 64, 1024, 4),
                                          (512, 512, 64, 1)])
def test_tn_weight_gradient(m, n, k, splits):
    torch.manual_seed(m + 7 * n + k)
    dy, x = rnd(k, m), rnd(k, n)
    out = G.mm_tn(dy, x, splits=splits)
    assert rel(out, dy.float().t() @ x.float()) < 1e-5


def test_tn_beta_accumulate_into_row_slice():
    torch.manual_seed(5)
    dy, x = rnd(4096, 512), rnd(4096, 768)
    full = torch.randn(3 * 512, 768, device=dev)
    before = full.clone()
    G.mm_tn(dy, x, out=full[512:1024], beta=1.0, splits=4)
    ref = before[512:1024] + dy.float().t() @ x.float()
    assert rel(full[512:1024], ref) < 1e-5
    assert torch.equal(full[:512], before[:512]) and torch.equal(full[1024:], before[1024:])


def test_tn_beta_accumulate_single_split():
    """beta = 1 with ONE split runs the ping-pong kernel itself (no reduce
    pass): its fp32 epilogue adds beta * C (it stored over C before round 5)."""
    torch.manual_seed(9)
    dy, x = rnd(1024, 512), rnd(1024, 768)
    full = torch.randn(3 * 512, 768, device=dev)
    before = full.clone()
    G.mm_tn(dy, x, out=full[512:1024], beta=1.0, splits=1)
    ref = before[512:1024] + dy.float().t() @ x.float()
    assert rel(full[512:1024], ref) < 1e-5
    assert torch.equal(full[:512], before[:512]) and torch.equal(full[1024:], before[1024:])


def _grouped(probs):
    import ctypes
    from mtts import _lib as L
    arr = (L.GemmArgs * len(probs))()
    for a, (dy, x, out, beta) in zip(arr, probs):
        a.m, a.n, a.k, a.layout, a.splits, a.out_dtype = dy.shape[1], x.shape[1], dy.shape[0], G.TN, 1, 0
        a.lda, a.ldb, a.ldc = dy.stride(0), x.stride(0), out.stride(0)
        a.a, a.b, a.c, a.beta = dy.data_ptr(), x.data_ptr(), out.data_ptr(), beta
    lib = L.lib()
    return lib.mtts_gemm_grouped(arr, len(probs), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def test_tn_grouped_matches_each_problem():
    """mtts_gemm_grouped: one C2 decoder layer's projection weight gradients
    (in_proj 4096x1024, out_proj 1024x2048, q and out 1024x1024 over 16384
    tokens, text K/V 2048x1024 over 1024 tokens, FFN 2048x1024 / 1024x2048)
    plus ragged ones, with row-slice outputs and beta = 1 accumulation, in
    ONE launch, against fp32 products of the same bf16 operands."""
    torch.manual_seed(11)
    T, Tt = 16384, 1024
    shapes = [(T, 4096, 1024), (T, 1024, 2048), (T, 1024, 1024), (Tt, 2048, 1024), (T, 2048, 1024),
              (T, 1024, 2048), (1088, 264, 520), (64, 8, 8)]
    probs, refs = [], []
    inproj = torch.randn(3 * 1024, 1024, device=dev)
    before = inproj.clone()
    for i, (k, m, n) in enumerate(shapes):
        dy, x = rnd(k, m, scale=0.5), rnd(k, n, scale=0.5)
        if i == 2:        # q rows of the packed MHA in-projection, accumulated
            out, beta = inproj[:1024], 1.0
            ref = before[:1024] + dy.float().t() @ x.float()
        elif i == 3:      # k/v rows of it, written
            out, beta = inproj[1024:], 0.0
            ref = dy.float().t() @ x.float()
        else:
            out, beta = torch.full((m, n), float("nan"), device=dev), 0.0
            ref = dy.float().t() @ x.float()
        probs.append((dy, x, out, beta))
        refs.append((out, ref))
    probs.sort(key=lambda t: -t[0].shape[0])
    assert _grouped(probs) == 0
    for i, (out, ref) in enumerate(refs):
        assert torch.isfinite(out).all(), i
        assert rel(out, ref) < 1e-5, i


def test_tn_grouped_rejects_bad_problems():
    dy, x = rnd(128, 256), rnd(128, 256)
    out = torch.empty(256, 256, device=dev)
    assert _grouped([(dy, x, out, 0.5)]) != 0          # beta must be 0 or 1
    assert _grouped([(rnd(100, 256), rnd(100, 256), out, 0.0)]) != 0   # k % 64
    assert _grouped([(dy, x, out, 0.0)] * 25) != 0     # at most 24 problems


def test_default_splits_fill_the_chip():
    assert G.tn_splits(4096, 1024, 16384) * 16 * 4 >= 256
    assert G.tn_splits(1024, 1024, 16384) == 16
    assert G.tn_splits(256, 256, 64) == 1
    assert G.tn_splits(2048, 1024, 1024) == 4     # C2 text K/V: 32 tiles, 1024 tokens
    assert G.tn_splits(4096, 1024, 16384) == 4 and G.tn_splits(1024, 2048, 16384) == 8


def test_refuses_unsupported_shapes():
    a, b = rnd(256, 100), rnd(256, 100)
    with pytest.raises(RuntimeError, match="multiple of 64"):
        G.mm_nt(a, b)
    a, b = rnd(256, 128), rnd(12, 128)
    with pytest.raises(RuntimeError, match="multiple of 8"):
        G.mm_nt(a, b)


def test_ffn_fused_matches_per_op_path():
    """FFNFn (GELU fused into the GEMM epilogues) vs linear + F.gelu + linear,
    outputs and every gradient, bf16 compute with fp32 master weights."""
    torch.manual_seed(6)
    B, T, d, dff = 2, 512, 256, 512
    w1 = (torch.randn(dff, d, device=dev) * d ** -0.5).requires_grad_()
    b1 = (torch.randn(dff, device=dev) * 0.1).requires_grad_()
    w2 = (torch.randn(d, dff, device=dev) * dff ** -0.5).requires_grad_()
    b2 = (torch.randn(d, device=dev) * 0.1).requires_grad_()
    h0 = torch.randn(B, T, d, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, T, d, device=dev).to(torch.bfloat16)
    outs = []
    for fused in (True, False):
        h = h0.clone().requires_grad_()
        for p in (w1, b1, w2, b2):
            p.grad = None
        with LIN.cast_scope([w1, b1, w2, b2], torch.bfloat16):
            y = LIN.FFNFn.apply(h, w1, b1, w2, b2) if fused else \
                LIN.linear(F.gelu(LIN.linear(h, w1, b1)), w2, b2)
            y.backward(dy)
        outs.append([y.detach(), h.grad] + [p.grad.clone() for p in (w1, b1, w2, b2)])
    names = ["y", "dh", "dW1", "db1", "dW2", "db2"]
    for nm, a, b in zip(names, outs[0], outs[1]):
        assert rel(a, b) < 2e-2, nm


@pytest.fixture(params=["pingpong", "narrow", "fourwave"])
def gemm_mode(request):
    """The ping-pong kernel (default), the single-group kernel with 8-byte
    epilogue stores (the fallback for 8-byte-aligned outputs; forced with the
    gemm_narrow override) or the four-wave 128x128-per-wave NT tile (gemm_tile
    override 2; TN problems keep the ping-pong kernel)."""
    from mtts import _lib as L
    with L.override(gemm_narrow=1 if request.param == "narrow" else None,
                    gemm_tile=2 if request.param == "fourwave" else None):
        yield request.param


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 128), (1000, 264, 192), (300, 1032, 1024),
                                   (37, 8, 64), (4096, 96, 2048), (1024, 2048, 320)])
def test_nt_four_wave_tile(m, n, k):
    """The four-wave tile at K = 2 .. 64 K-steps of 32 (K = 64: the prologue's
    re-staged steps and the stale-slot reads past the end), ragged M / N
    edges, every epilogue."""
    from mtts import _lib as L
    torch.manual_seed(m + 3 * n + k)
    a, b = rnd(m, k), rnd(n, k)
    ref = a.float() @ b.float().t()
    with L.override(gemm_tile=2):
        assert rel(G.mm_nt(a, b), ref) < 1e-2
        bias = rnd(n, dtype=torch.float32)
        assert rel(G.mm_nt(a, b, bias=bias), ref + bias) < 1e-2
        pre = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        act = G.mm_nt(a, b, bias=bias, gelu_aux=pre)
        assert rel(pre, ref + bias) < 1e-2 and gelu_matches(act, pre)
        aux = rnd(m, n, scale=3.0)
        g = G.mm_nt(a, b, dgelu_aux=aux)
        assert rel(g, torch.ops.aten.gelu_backward(ref.to(torch.bfloat16), aux)) < 1e-2


@pytest.mark.parametrize("m,n,k", [(16384, 4096, 1024), (16484, 4104, 1024), (4096, 2048, 128), (8192, 1024, 2048)])
def test_nt_every_kernel_many_tiles(gemm_mode, m, n, k):
    """More work items than CUs (several rounds of workgroups), ragged edges
    in both dimensions, K of 2 K-tiles; plain, bias + GELU and GELU-backward."""
    torch.manual_seed(m + n + k)
    a, b = rnd(m, k), rnd(n, k)
    ref = a.float() @ b.float().t()
    assert rel(G.mm_nt(a, b), ref) < 1e-2
    bias = rnd(n, dtype=torch.float32)
    pre = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    act = G.mm_nt(a, b, bias=bias, gelu_aux=pre)
    assert rel(pre, ref + bias) < 1e-2
    assert gelu_matches(act, pre)
    bias16 = rnd(n)
    assert rel(G.mm_nt(a, b, bias=bias16), ref + bias16.float()) < 1e-2
    aux = rnd(m, n, scale=3.0)
    g = G.mm_nt(a, b, dgelu_aux=aux)
    assert rel(g, torch.ops.aten.gelu_backward(ref.to(torch.bfloat16), aux)) < 1e-2


def test_nt_every_kernel_strided_output(gemm_mode):
    torch.manual_seed(11)
    a, b = rnd(9000, 512), rnd(1032, 512)
    out_full = torch.zeros(9000, 1048, device=dev, dtype=torch.bfloat16)
    out = out_full[:, 8:8 + 1032]
    G.mm_nt(a, b, out=out)
    assert rel(out, a.float() @ b.float().t()) < 1e-2
    assert out_full[:, :8].abs().max() == 0 and out_full[:, 1040:].abs().max() == 0


@pytest.mark.parametrize("m,n,k,splits", [(1024, 1024, 16384, 32), (2056, 1032, 8192, 4), (4096, 1024, 16384, 4)])
def test_tn_every_kernel_many_items(gemm_mode, m, n, k, splits):
    torch.manual_seed(m + n + k + splits)
    dy, x = rnd(k, m), rnd(k, n)
    out = G.mm_tn(dy, x, splits=splits)
    assert rel(out, dy.float().t() @ x.float()) < 1e-5


# ---------------------------------------------------------------- skinny GEMMs (csrc/skinny.hip)
@pytest.mark.parametrize("m,n,k", [(16384, 96, 2048), (16384, 64, 2048), (1000, 96, 2048), (37, 36, 128),
                                   (130, 128, 96), (64, 4, 32), (513, 100, 4096)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_skinny_n(m, n, k, out_dtype):
    """SKINNY_N (n <= 128: x_proj forward, dt_proj data gradient) vs the fp32
    product of the same bf16 operands; ragged m and n, K split over 4 waves."""
    torch.manual_seed(m + n + k)
    a, b = rnd(m, k), rnd(n, k)
    assert G.skinny_ok(a, b)
    out = G.mm_skinny(a, b, out_dtype=out_dtype)
    ref = a.float() @ b.float().t()
    assert rel(out, ref) < (1e-2 if out_dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("m,n,k", [(16384, 2048, 64), (16384, 2048, 96), (1000, 520, 64), (77, 256, 128),
                                   (64, 200, 32)])
def test_skinny_small_k(m, n, k):
    """SMALL_K (k <= 128: dt_proj forward) vs fp32 of the same operands."""
    torch.manual_seed(m + n + k + 1)
    a, b = rnd(m, k), rnd(n, k)
    out = G.mm_skinny(a, b)
    assert rel(out, a.float() @ b.float().t()) < 1e-2


def test_skinny_strided_views_and_accumulate():
    """The decoder's operand layouts: dt = x_dbl[:, :64] (row stride 96) for
    the dt_proj forward; d(dt) written as fp32 into the d(x_dbl)[:, :64] slice;
    du += d(x_dbl) W_x accumulated in place (beta = 1, bf16 du) -- the rest of
    each row untouched."""
    torch.manual_seed(7)
    m, di, r = 2048, 2048, 64
    x_dbl = rnd(m, r + 32)
    wdt = rnd(di, r)
    delta = G.mm_skinny(x_dbl[:, :r], wdt)
    assert rel(delta, x_dbl[:, :r].float() @ wdt.float().t()) < 1e-2
    dd = rnd(m, di)
    dx = torch.full((m, r + 32), 7.0, device=dev)
    wdt_t = wdt.t().contiguous()
    G.mm_skinny(dd, wdt_t, out=dx[:, :r])
    assert rel(dx[:, :r], dd.float() @ wdt.float()) < 1e-5
    assert (dx[:, r:] == 7.0).all()
    gx = rnd(m, r + 32)
    wx_t = rnd(di, r + 32)
    du = rnd(m, di)
    ref = (du.float() + gx.float() @ wx_t.float().t())
    G.mm_skinny(gx, wx_t, out=du, beta=1.0)
    assert rel(du, ref) < 1e-2


@pytest.mark.parametrize("n", [132, 260, 264])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_skinny_small_k_ragged_columns(n, beta):
    """SMALL_K's bf16 stores move 8 columns per lane: n % 8 == 4 with a bf16
    C is refused (skinny_ok and the C-ABI), never written past the row end;
    fp32 C (4-column stores) takes n % 4 == 0, with and without accumulate."""
    torch.manual_seed(n + int(beta))
    m, k = 200, 64
    a, b = rnd(m, k), rnd(n, k)
    if n % 8:
        assert not G.skinny_ok(a, b, out_dtype=torch.bfloat16)
        with pytest.raises(RuntimeError, match="SMALL_K with bf16 C"):
            G.mm_skinny(a, b, out_dtype=torch.bfloat16)
    else:
        assert G.skinny_ok(a, b, out_dtype=torch.bfloat16)
        # a 16-row guard band past C: nothing outside the (m, n) block changes
        buf = torch.full((m + 16, n), 3.0, device=dev, dtype=torch.bfloat16)
        c = buf[:m]
        c0 = c.float().clone()
        G.mm_skinny(a, b, out=c, beta=beta)
        assert rel(c, a.float() @ b.float().t() + beta * c0) < 1e-2
        assert (buf[m:] == 3.0).all()
    c32 = torch.full((m, n), 0.5, device=dev)
    ref = a.float() @ b.float().t() + beta * c32
    assert G.skinny_ok(a, b, out_dtype=torch.float32, out=c32)
    G.mm_skinny(a, b, out=c32, beta=beta)
    assert rel(c32, ref) < 1e-5


def test_skinny_rejects_bad_shapes():
    a, b = rnd(64, 48), rnd(32, 48)
    assert not G.skinny_ok(a, b)                     # k % 32
    a, b = rnd(64, 256), rnd(200, 256)
    assert not G.skinny_ok(a, b)                     # n > 128 and k > 128
    with pytest.raises(RuntimeError, match="gemm_skinny"):
        G.mm_skinny(a, b)


@pytest.mark.parametrize("shape", [(96, 2048), (2048, 64)])
def test_tn_skinny_weight_gradients(shape):
    """x_proj / dt_proj weight gradients (one output dim 64-96) on the TN
    kernel, split-K: dW = dy^T x in fp32."""
    torch.manual_seed(11)
    M = 16384
    dy, x = rnd(M, shape[0]), rnd(M, shape[1])
    out = LIN.wgrad(dy, x)
    ref = dy.float().t() @ x.float()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("k,m,n,trans", [(16384, 2048, 64, False), (16384, 2048, 96, True), (1000, 256, 40, False),
                                         (77, 128, 8, True), (4096, 384, 128, False)])
def test_skinny_tn_weight_gradient(k, m, n, trans):
    """SKINNY_TN (x_proj / dt_proj weight gradients): fp32 a^T b over k
    token rows (ragged k, n < 16 * blocks), or its transpose, vs fp32 torch;
    the narrow operand as a strided column slice like x_dbl[:, :dt_rank]."""
    torch.manual_seed(k + m + n)
    a = rnd(k, m)
    bb = rnd(k, n + 32)
    b = bb[:, :n]
    assert G.skinny_tn_ok(a, b)
    out = G.mm_skinny_tn(a, b, trans_c=trans)
    ref = a.float().t() @ b.float()
    if trans:
        ref = ref.t()
    assert out.shape == ref.shape
    assert rel(out, ref) < 1e-5


# ------------------------------------------------------------------ C2 routing, every hand-written mode
C2_M = 16384


@pytest.mark.parametrize("ragged", [False, True])
def test_c2_projection_route_every_hand_written_kernel(ragged):
    """Every GEMM a C2 layer routes to the hand-written kernels (linear.proj /
    FFN epilogues / linear.wgrad at the default tn_splits), at C2's token count
    (and ragged: 56 rows fewer, an output width off the 256 tile), bf16
    operands, against fp32 products of the same operands: bf16 outputs 1e-2 of
    max, fp32 weight gradients (split-K, fixed-order slab sum) 1e-5."""
    torch.manual_seed(17 + int(ragged))
    M = C2_M - (56 if ragged else 0)
    dn = 8 if ragged else 0
    nt_cases = {   # name: (n, k, epilogue)
        "in_proj fwd": (4096 + dn, 1024, None), "in_proj dgrad": (1024 + dn, 4096, None),
        "out_proj fwd": (1024 + dn, 2048, None), "out_proj dgrad": (2048 + dn, 1024, None),
        "q / o fwd + bias": (1024 + dn, 1024, "bias"), "FFN1 + bias + GELU": (2048 + dn, 1024, "gelu"),
        "FFN2 fwd + bias": (1024 + dn, 2048, "bias"), "FFN2 dgrad + GELU'": (2048 + dn, 1024, "dgelu"),
    }
    for name, (n, k, epi) in nt_cases.items():
        x, w = rnd(M, k), rnd(n, k)
        assert LIN._nt_route(x, w), name
        ref = x.float() @ w.float().t()
        if epi is None:
            got = LIN.proj(x, w)
            assert rel(got, ref) < 1e-2, name
        elif epi == "bias":
            b = rnd(n, dtype=torch.float32)
            assert rel(LIN.proj(x, w, b), ref + b) < 1e-2, name
        elif epi == "gelu":
            b = rnd(n, dtype=torch.float32)
            pre = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
            act = G.mm_nt(x, w, bias=b, gelu_aux=pre)
            assert rel(pre, ref + b) < 1e-2, name
            assert gelu_matches(act, pre), name
        else:
            aux = rnd(M, n, scale=3.0)
            got = G.mm_nt(x, w, dgelu_aux=aux)
            assert rel(got, torch.ops.aten.gelu_backward(ref.to(torch.bfloat16), aux)) < 1e-2, name
    tn_cases = {"in_proj": (4096 + dn, 1024), "out_proj": (1024 + dn, 2048), "q / o": (1024 + dn, 1024),
                "FFN1": (2048 + dn, 1024), "FFN2": (1024 + dn, 2048)}
    for name, (m, n) in tn_cases.items():
        # the token axis is the reduction (k % (64 * splits)): C2's full count,
        # ragged only in the output dims
        dy, x = rnd(C2_M, m), rnd(C2_M, n)
        splits = G.tn_splits(m, n, C2_M)
        assert G.tn_ok(dy, x) and LIN.HIP_WGRAD_MIN <= min(m, n), name
        assert splits > 1, f"{name}: C2 weight gradients run split-K"
        got = LIN.wgrad(dy, x)
        assert rel(got, dy.float().t() @ x.float()) < 1e-5, f"{name} (splits {splits})"
        # the default split count also into a row slice with accumulate (beta = 1)
        full = torch.randn(m + 16, n, device=dev)
        before = full.clone()
        G.mm_tn(dy, x, out=full[8:8 + m], beta=1.0)
        assert rel(full[8:8 + m], before[8:8 + m] + dy.float().t() @ x.float()) < 1e-5, f"{name} beta"
        assert torch.equal(full[:8], before[:8]) and torch.equal(full[8 + m:], before[8 + m:]), name
