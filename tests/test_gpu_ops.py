"""GPU parity of the libmtts kernels against the golden vectors (HF's
independent Mamba v1, float64) and the CPU oracle.  Tolerance: the north
star's 1e-3 relative (fp32), measured as max|err| <= 1e-3 * max|ref| per
tensor; bf16 I/O runs use a looser, stated bound."""

import numpy as np
import pytest
import torch

from oracle import mamba_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 1e-3


def close(out, ref, rtol=RTOL, name=""):
    out = torch.as_tensor(out).detach().double().cpu()
    ref = torch.as_tensor(np.asarray(ref) if not torch.is_tensor(ref) else ref).double().cpu()
    assert out.shape == ref.shape, f"{name}: shape {tuple(out.shape)} vs {tuple(ref.shape)}"
    assert torch.isfinite(out).all(), f"{name}: non-finite"
    err = (out - ref).abs().max().item()
    scale = max(ref.abs().max().item(), 1e-6)
    assert err <= rtol * scale, f"{name}: max|err|={err:.3e} > {rtol}*{scale:.3e}"


def cl(a, dtype=torch.float32):
    """(B, D, L) numpy -> channel-last (B, L, D) cuda tensor"""
    return torch.from_numpy(np.ascontiguousarray(np.swapaxes(a, 1, 2))).to(DEV, dtype)


def g32(a):
    return torch.from_numpy(np.asarray(a)).to(DEV, torch.float32)


@pytest.fixture(params=["2", "4", "4:s3", "4n", "2n:s2", "4c1"])
def scan_p(request):
    """P (lanes per channel) and, with ':sK', a forced split of L into K
    segments for both the forward and the backward (two-pass path); 'n'
    forces the narrow (per-lane element) forward kernel instead of the
    16-byte-chunk LDS-DMA one; 'c1' the one-lane-per-channel forward
    (scan_fwd_c1_kernel) below its B*D threshold wherever D % 64 == 0.
    Forced through the library's kernel-path overrides (mtts_set_override)."""
    from mtts import _lib as L
    p, _, segs = request.param.partition(":s")
    path = None
    if p.endswith("c1"):
        p, path = p[:-2], L.SCAN_C1
    if p.endswith("n"):
        p, path = p[:-1], L.SCAN_NARROW
    with L.override(scan_p=int(p), scan_path=path, scan_segs=int(segs) if segs else None,
                    scan_bwd_segs=int(segs) if segs else None):
        yield request.param


@pytest.mark.parametrize("name", ["scan_full.npz", "scan_plain.npz", "scan_short.npz"])
def test_scan_fwd_bwd_vs_golden(golden, name, scan_p):
    from mtts import ops
    g = golden(name)
    sp = bool(g["softplus"])
    u, delta, z = cl(g["u"]), cl(g["delta"]), cl(g["z"]) if "z" in g else None
    Bm, Cm = cl(g["B"]), cl(g["C"])
    A = g32(g["A"])
    D = g32(g["D"]) if "D" in g else None
    bias = g32(g["delta_bias"]) if "delta_bias" in g else None
    out, last, ckpt = ops.scan_fwd(u, delta, A, Bm, Cm, D, z, bias, sp, want_last=True, want_ckpt=True)
    close(out.transpose(1, 2), g["out"], name="out")
    close(last, g["last_state"], name="last_state")
    du, dd, dz, dB, dC, dA, dD, db, _ = ops.scan_bwd(u, delta, A, Bm, Cm, D, z, bias, sp, None, ckpt, cl(g["dout"]))
    close(du.transpose(1, 2), g["du"], name="du")
    close(dd.transpose(1, 2), g["ddelta"], name="ddelta")
    close(dB.transpose(1, 2), g["dB"], name="dB")
    close(dC.transpose(1, 2), g["dC"], name="dC")
    close(dA, g["dA"], name="dA")
    if z is not None:
        close(dz.transpose(1, 2), g["dz"], name="dz")
    if D is not None:
        close(dD, g["dD"], name="dD")
    if bias is not None:
        close(db, g["ddelta_bias"], name="ddelta_bias")


@pytest.mark.parametrize("shape", [(1, 1, 1), (2, 3, 5), (3, 100, 37), (2, 70, 130), (1, 64, 1000), (2, 200, 77),
                                   (1, 136, 300)])
def test_scan_ragged_shapes_and_h0_split(shape, scan_p):
    """Ragged (B, D, L) incl. L=1, D not a multiple of 64, L not a multiple of
    16; and scanning [0,L1) then [L1,L) from h0=last_state equals one scan."""
    from mtts import ops
    torch.manual_seed(sum(shape))
    B, D, L = shape
    u = torch.randn(B, L, D, device=DEV)
    dl = torch.randn(B, L, D, device=DEV) * 0.5
    z = torch.randn(B, L, D, device=DEV)
    A = -torch.exp(torch.randn(D, 16, device=DEV) * 0.5)
    Bm = torch.randn(B, L, 16, device=DEV)
    Cm = torch.randn(B, L, 16, device=DEV)
    Dp = torch.randn(D, device=DEV)
    bias = torch.randn(D, device=DEV) * 0.1
    out, last, _ = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True)
    ref, rlast = R.selective_scan_ref(*(t.double().cpu() for t in (u.transpose(1, 2), dl.transpose(1, 2), A,
                                                                  Bm.transpose(1, 2), Cm.transpose(1, 2), Dp,
                                                                  z.transpose(1, 2), bias)),
                                      delta_softplus=True, return_last_state=True)
    close(out.transpose(1, 2), ref, name="out")
    close(last, rlast, name="last")
    if L > 1:
        L1 = L // 2
        o1, l1, _ = ops.scan_fwd(u[:, :L1], dl[:, :L1], A, Bm[:, :L1].contiguous(), Cm[:, :L1].contiguous(), Dp,
                                 z[:, :L1], bias, True, want_last=True)
        o2, l2, _ = ops.scan_fwd(u[:, L1:], dl[:, L1:], A, Bm[:, L1:].contiguous(), Cm[:, L1:].contiguous(), Dp,
                                 z[:, L1:], bias, True, h0=l1, want_last=True)
        close(torch.cat([o1, o2], 1), out, rtol=1e-5, name="split-out")
        close(l2, last, rtol=1e-5, name="split-last")


def _scan_inputs(B, L, D, dtype, bc_dtype, seed, strided_bc=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    u = torch.randn(B, L, D, device=DEV, generator=g).to(dtype)
    z = torch.randn(B, L, D, device=DEV, generator=g).to(dtype)
    dl = (torch.randn(B, L, D, device=DEV, generator=g) * 0.5).to(dtype)
    if strided_bc:  # B / C as column slices of an x_proj-style (B, L, R + 2N) row, as the decoder passes them
        xd = torch.randn(B, L, 64 + 32, device=DEV, generator=g).to(bc_dtype)
        Bm, Cm = xd[..., 64:80], xd[..., 80:96]
    else:
        Bm = torch.randn(B, L, 16, device=DEV, generator=g).to(bc_dtype)
        Cm = torch.randn(B, L, 16, device=DEV, generator=g).to(bc_dtype)
    A = -torch.exp(torch.randn(D, 16, device=DEV, generator=g) * 0.5)
    Dp = torch.randn(D, device=DEV, generator=g)
    bias = torch.randn(D, device=DEV, generator=g) * 0.1
    h0 = torch.randn(B, D, 16, device=DEV, generator=g) * 0.5
    return u, dl, A, Bm, Cm, Dp, z, bias, h0


def _with_path(path, fn):
    """Run fn with the scan forward path forced (None: automatic)."""
    from mtts import _lib as L
    with L.override(scan_path=path):
        return fn()


@pytest.mark.parametrize("B,L,D", [(1, 1, 64), (2, 37, 128), (3, 200, 192), (2, 1003, 64), (1, 16, 320), (2, 203, 256),
                                   (1, 50, 512), (1, 1, 256), (3, 1003, 512), (1, 17, 768)])
@pytest.mark.parametrize("io,bc", [("f32", "f32"), ("f32", "bf16"), ("bf16", "bf16"), ("bf16", "f32")])
@pytest.mark.parametrize("with_z,strided", [(True, False), (False, True)])
def test_scan_c1_kernel_vs_oracle(B, L, D, io, bc, with_z, strided):
    """scan_fwd_c1_kernel (forced) against the float64 oracle on the same
    (already rounded) inputs: outputs, last state and the backward's
    checkpoints (h every 16 steps, compared with the P=4 LDS-DMA kernel's);
    h0, ragged L (tail tiles), D % 256 != 0 (idle waves), strided B/C."""
    from mtts import _lib, ops
    kernel = "c1"
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}
    u, dl, A, Bm, Cm, Dp, z, bias, h0 = _scan_inputs(B, L, D, dt[io], dt[bc], B * L + D, strided)
    z = z if with_z else None
    run = lambda: ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, h0=h0, want_last=True,  # noqa: E731
                               want_ckpt=True)
    out, last, ck = _with_path(_lib.SCAN_C1, run)
    out_w, last_w, ck_w = _with_path(2, run)   # the P-lane LDS-DMA kernel
    ref, rlast = R.selective_scan_ref(*(t.double().cpu() for t in (u.transpose(1, 2), dl.transpose(1, 2), A,
                                                                  Bm.transpose(1, 2), Cm.transpose(1, 2), Dp)),
                                      None if z is None else z.double().cpu().transpose(1, 2),
                                      bias.double().cpu(), delta_softplus=True, return_last_state=True,
                                      h0=h0.double().cpu())
    tol = RTOL if io == "f32" else 1e-2  # bf16 output rounding
    close(out.transpose(1, 2), ref, rtol=tol, name=f"{kernel} out")
    close(last, rlast, name=f"{kernel} last")
    close(ck, ck_w, rtol=1e-5, name=f"{kernel} ckpt vs w2")
    close(out.float(), out_w.float(), rtol=tol, name=f"{kernel} vs w2 out")


@pytest.mark.parametrize("path,segs", [(1, None), (2, None), (2, 3), (3, None)])
@pytest.mark.parametrize("L", [37, 1003])
@pytest.mark.parametrize("io", ["f32", "bf16"])
def test_scan_rows_past_L_neither_read_nor_written(path, segs, L, io):
    """The buffer-addressed forward kernels (c1, the P-lane LDS-DMA kernel)
    and the narrow kernel on row views of larger tensors: rows >= L of u /
    delta / z / B / C hold NaN and the output rows >= L hold a sentinel.  The
    outputs must equal the run on contiguous copies bit for bit, stay finite,
    and the sentinel rows must be untouched (no tile row past L is used or
    stored, whatever the buffer range check does with the scalar offset)."""
    from mtts import _lib, ops
    B, D, pad = 2, 512, 40
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}[io]
    u, dl, A, Bm, Cm, Dp, z, bias, h0 = _scan_inputs(B, L, D, dt, dt, L + path)

    def big(t, fill):
        bt = torch.full((t.shape[0], L + pad, t.shape[2]), fill, device=DEV, dtype=t.dtype)
        bt[:, :L] = t
        return bt

    nan = float("nan")
    ub, db_, zb, Bb, Cb = big(u, nan), big(dl, nan), big(z, nan), big(Bm, nan), big(Cm, nan)
    ob = torch.full((B, L + pad, D), 7.0, device=DEV, dtype=dt)
    with _lib.override(scan_path=path, scan_segs=segs):
        ref, rlast, _ = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, h0=h0, want_last=True)
        out, last, _ = ops.scan_fwd(ub[:, :L], db_[:, :L], A, Bb[:, :L], Cb[:, :L], Dp, zb[:, :L], bias, True,
                                    h0=h0, want_last=True, out=ob[:, :L])
    assert torch.isfinite(out).all() and torch.isfinite(last).all()
    assert torch.equal(out, ref) and torch.equal(last, rlast)
    assert (ob[:, L:] == 7.0).all(), "a store landed past row L"


def test_scan_c1_north_star_width():
    """At the north-star width (B=32, D=2048: the c1 kernel is the default)
    with a shorter L: c1 against the P=4 LDS-DMA kernel on every element, and
    against the float64 oracle on a 64-channel slice of two batch rows."""
    from mtts import ops
    B, L, D = 32, 520, 2048
    u, dl, A, Bm, Cm, Dp, z, bias, _ = _scan_inputs(B, L, D, torch.float32, torch.float32, 7)
    dl = dl * 0.2
    run = lambda: ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True)  # noqa: E731
    out, last, _ = _with_path(None, run)
    out_w, last_w, _ = _with_path(2, run)
    close(out, out_w, rtol=1e-5, name="c1 vs w2 out")
    close(last, last_w, rtol=1e-5, name="c1 vs w2 last")
    for b, c in ((0, 0), (31, 1984)):
        sl = lambda t: t[b:b + 1, :, c:c + 64].double().cpu().transpose(1, 2)  # noqa: E731
        ref = R.selective_scan_ref(sl(u), sl(dl), A[c:c + 64].double().cpu(),
                                   Bm[b:b + 1].double().cpu().transpose(1, 2),
                                   Cm[b:b + 1].double().cpu().transpose(1, 2), Dp[c:c + 64].double().cpu(), sl(z),
                                   bias[c:c + 64].double().cpu(), delta_softplus=True)
        close(out[b:b + 1, :, c:c + 64].transpose(1, 2), ref, name=f"c1 oracle slice b={b} c={c}")


def test_scan_bf16_io(golden):
    """bf16 u/delta/z/B/C/out with fp32 math: bounded by bf16 input rounding."""
    from mtts import ops
    g = golden("scan_full.npz")
    bf = torch.bfloat16
    out, _, _ = ops.scan_fwd(cl(g["u"], bf), cl(g["delta"], bf), g32(g["A"]), cl(g["B"], bf), cl(g["C"], bf),
                             g32(g["D"]), cl(g["z"], bf), g32(g["delta_bias"]), True)
    ref = R.selective_scan_ref(*(torch.from_numpy(g[k]).to(bf).double() for k in ("u", "delta")),
                               torch.from_numpy(g["A"]).double(),
                               *(torch.from_numpy(g[k]).to(bf).double() for k in ("B", "C")),
                               torch.from_numpy(g["D"]).double(), torch.from_numpy(g["z"]).to(bf).double(),
                               torch.from_numpy(g["delta_bias"]).double(), True)
    close(out.transpose(1, 2), ref, rtol=1e-2, name="bf16 out")


def test_scan_deterministic():
    from mtts import ops
    torch.manual_seed(0)
    B, L, D = 2, 300, 256
    args = [torch.randn(B, L, D, device=DEV), torch.randn(B, L, D, device=DEV) * 0.3,
            -torch.rand(D, 16, device=DEV) - 0.1, torch.randn(B, L, 16, device=DEV), torch.randn(B, L, 16, device=DEV)]
    o1, _, ck = ops.scan_fwd(*args, want_ckpt=True)
    o2, _, _ = ops.scan_fwd(*args)
    assert torch.equal(o1, o2)
    g = torch.randn(B, L, D, device=DEV)
    r1 = ops.scan_bwd(*args, None, None, None, True, None, ck, g)
    r2 = ops.scan_bwd(*args, None, None, None, True, None, ck, g)
    for a, b in zip(r1, r2):
        if a is not None:
            assert torch.equal(a, b)


def test_conv1d_fwd_bwd_update_vs_golden(golden):
    from mtts import ops
    g = golden("conv1d.npz")
    x = cl(g["x"])
    w, b = g32(g["w"]), g32(g["b"])
    out, st = ops.conv_fwd(x, w, b, True, want_state=True)
    close(out.transpose(1, 2), g["out"], name="conv out")
    close(st, g["x"][:, :, -4:], name="conv state")
    dx, dw, db = ops.conv_bwd(x, w, b, cl(g["dout"]), True)
    close(dx.transpose(1, 2), g["dx"], name="dx")
    close(dw, g["dw"], name="dw")
    close(db, g["db"], name="db")
    xs = torch.from_numpy(g["xs"]).to(DEV)
    state = torch.zeros(2, 64, 4, device=DEV)
    outs = [ops.conv_update(xs[:, :, t].contiguous(), state, w, b, True) for t in range(xs.shape[-1])]
    close(torch.stack(outs, -1), g["upd_out"], name="update out")
    close(state, g["upd_state"], name="update state")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(1, 1, 8), (2, 37, 24), (2, 100, 512), (1, 33, 2048)])
def test_conv1d_shapes_strided_and_prefix_state(shape, dtype):
    """strided input view (xz[..., :D]), conv_state_in prefix == running on the
    concatenated sequence, ragged L."""
    from mtts import ops
    torch.manual_seed(1)
    B, L, D = shape
    xz = torch.randn(B, L + 6, 2 * D, device=DEV).to(dtype)
    x = xz[:, 6:, :D]
    prefix = xz[:, :6, :D]
    w = torch.randn(D, 4, device=DEV)
    b = torch.randn(D, device=DEV)
    _, st = ops.conv_fwd(prefix, w, b, True, want_state=True)
    out, st2 = ops.conv_fwd(x, w, b, True, state_in=st, want_state=True)
    full, stf = ops.conv_fwd(xz[:, :, :D], w, b, True, want_state=True)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(out.float(), full[:, 6:].float(), rtol=tol, name="prefix")
    close(st2, stf, rtol=1e-6, name="state")
    ref, _ = R.causal_conv1d_ref(x.transpose(1, 2).double().cpu(), w.double().cpu(), b.double().cpu(), "silu",
                                 st.double().cpu())
    close(out.transpose(1, 2).float(), ref, rtol=tol, name="vs oracle")
    go = torch.randn(B, L, D, device=DEV).to(dtype)
    dx, dw, db = ops.conv_bwd(xz[:, 6:, :D].contiguous(), w, b, go, True)
    xr = x.transpose(1, 2).double().cpu().requires_grad_(True)
    wr, br = w.double().cpu().requires_grad_(True), b.double().cpu().requires_grad_(True)
    o, _ = R.causal_conv1d_ref(xr, wr, br, "silu")
    (o * go.transpose(1, 2).double().cpu()).sum().backward()
    close(dx.transpose(1, 2).float(), xr.grad, rtol=tol, name="dx")
    close(dw, wr.grad, rtol=tol, name="dw")
    close(db, br.grad, rtol=tol, name="db")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 2048, 2048), (1, 71, 256), (3, 130, 64)])
def test_conv1d_tiled_vs_oracle_with_state(shape, dtype):
    """Tiled conv kernels (all tile loads in flight; 8-wave backward with an
    LDS sum of the time tiles' dw/db) on the in_proj layout (x = xz[..., :D],
    row stride 2D), ragged L, a prefilled conv_state entering the forward AND
    the backward (pre-activations and dw include the history), vs the float64
    oracle; the untiled kernels (override conv_untiled) give the same values."""
    from mtts import _lib
    from mtts import ops
    torch.manual_seed(2)
    B, L, D = shape
    xz = torch.randn(B, L, 2 * D, device=DEV).to(dtype)
    x = xz[..., :D]
    w = torch.randn(D, 4, device=DEV) * 0.5
    b = torch.randn(D, device=DEV) * 0.1
    st = torch.randn(B, D, 4, device=DEV)
    out, st_out = ops.conv_fwd(x, w, b, True, state_in=st, want_state=True)
    xr = x.transpose(1, 2).double().cpu().requires_grad_(True)
    wr, br = w.double().cpu().requires_grad_(True), b.double().cpu().requires_grad_(True)
    ref, _ = R.causal_conv1d_ref(xr, wr, br, "silu", st.double().cpu())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(out.transpose(1, 2).float(), ref.detach(), rtol=tol, name="fwd vs oracle")
    go = torch.randn(B, L, D, device=DEV).to(dtype)
    dxz = torch.zeros_like(xz)
    _, dw, db = ops.conv_bwd(x, w, b, go, True, dx=dxz[..., :D], state_in=st)
    (ref * go.transpose(1, 2).double().cpu()).sum().backward()
    close(dxz[..., :D].transpose(1, 2).float(), xr.grad, rtol=tol, name="dx")
    assert dxz[..., D:].abs().max().item() == 0.0, "dx wrote outside its half of d(xz)"
    close(dw, wr.grad, rtol=tol, name="dw")
    close(db, br.grad, rtol=tol, name="db")
    with _lib.override(conv_untiled=1):
        out2, _ = ops.conv_fwd(x, w, b, True, state_in=st, want_state=True)
        dxz2 = torch.zeros_like(xz)
        _, dw2, db2 = ops.conv_bwd(x, w, b, go, True, dx=dxz2[..., :D], state_in=st)
    assert torch.equal(out, out2), "tiled and untiled forward differ"
    assert torch.equal(dxz, dxz2), "tiled and untiled dx differ"
    close(dw2, dw, rtol=1e-5, name="dw tiled vs untiled")
    close(db2, db, rtol=1e-5, name="db tiled vs untiled")


@pytest.mark.parametrize("untiled", [0, 1])
@pytest.mark.parametrize("with_state", [False, True])
@pytest.mark.parametrize("L,D", [(37, 64), (130, 2048), (1003, 200)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv1d_rows_outside_0_L_neither_read_nor_written(dtype, L, D, with_state, untiled):
    """The buffer-addressed tiled conv kernels put a tile's row origin in the
    scalar offset, so their first tile issues loads for rows -3..-1 and their
    last tile rows past L (read as 0 by the range check, which covers voffset +
    soffset: profiles/r05_buffer_oob_probe.txt).  Here x / dout are row views
    of larger tensors whose rows before 0 and from L on hold NaN, and out / dx
    are row views of sentinel-filled tensors: results must equal the run on
    contiguous copies bit for bit, stay finite, and the sentinel rows must be
    untouched.  Channel-last with the in_proj row stride (2D), D % 256 != 0
    cases included (partial channel blocks)."""
    from mtts import _lib, ops
    torch.manual_seed(5)
    B, pad = 2, 24
    nan = float("nan")
    w = torch.randn(D, 4, device=DEV) * 0.5
    b = torch.randn(D, device=DEV) * 0.1
    st = torch.randn(B, D, 4, device=DEV) if with_state else None
    xz = torch.randn(B, L, 2 * D, device=DEV).to(dtype)
    go = torch.randn(B, L, D, device=DEV).to(dtype)

    def poisoned(t, fill):
        bt = torch.full((t.shape[0], L + 2 * pad, t.shape[2]), fill, device=DEV, dtype=t.dtype)
        bt[:, pad:pad + L] = t
        return bt

    xzb, gob = poisoned(xz, nan), poisoned(go, nan)
    ob = torch.full((B, L + 2 * pad, D), 7.0, device=DEV, dtype=dtype)
    dxb = torch.full((B, L + 2 * pad, 2 * D), 7.0, device=DEV, dtype=dtype)
    with _lib.override(conv_untiled=untiled):
        ref, _ = ops.conv_fwd(xz[..., :D], w, b, True, state_in=st, want_state=True)
        dref = torch.zeros_like(xz)
        _, dwr, dbr = ops.conv_bwd(xz[..., :D], w, b, go, True, dx=dref[..., :D], state_in=st)
        out, _ = ops.conv_fwd(xzb[:, pad:pad + L, :D], w, b, True, state_in=st, want_state=True,
                              out=ob[:, pad:pad + L])
        _, dw, db = ops.conv_bwd(xzb[:, pad:pad + L, :D], w, b, gob[:, pad:pad + L], True,
                                 dx=dxb[:, pad:pad + L, :D], state_in=st)
    assert torch.isfinite(out).all() and torch.isfinite(dw).all() and torch.isfinite(db).all()
    assert torch.equal(out, ref)
    assert torch.equal(dxb[:, pad:pad + L, :D], dref[..., :D])
    assert torch.equal(dw, dwr) and torch.equal(db, dbr)
    assert (ob[:, :pad] == 7.0).all() and (ob[:, pad + L:] == 7.0).all(), "a conv store landed outside [0, L)"
    assert (dxb[:, :pad] == 7.0).all() and (dxb[:, pad + L:] == 7.0).all(), "a dx store landed outside [0, L)"
    assert (dxb[..., D:] == 7.0).all(), "dx wrote outside its half"


def test_state_update_vs_golden(golden):
    from mtts import ops
    g = golden("state_update.npz")
    A, D, bias = g32(g["A"]), g32(g["D"]), g32(g["delta_bias"])
    st = torch.zeros(2, 32, 16, device=DEV)
    outs = []
    for t in range(g["u"].shape[-1]):
        sl = lambda k: torch.from_numpy(np.ascontiguousarray(g[k][..., t])).to(DEV)  # noqa: E731
        outs.append(ops.state_update(st, sl("u"), sl("delta"), A, sl("B"), sl("C"), D, sl("z"), bias, True))
    close(torch.stack(outs, -1), g["step_out"], name="step out")
    close(st, g["step_state"], name="step state")
    close(torch.stack(outs, -1), g["full_out"], name="step == full scan")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols,rows,film", [(64, 6, False), (1024, 64, True), (512, 40, True), (2048, 17, False),
                                            (512, 1024, False), (256, 3001, False),
                                            (96 * 2, 5, False)])
def test_layernorm_res_film_fwd_bwd(dtype, cols, rows, film):
    from mtts import ops
    torch.manual_seed(cols + rows)
    G = 2 if (film and rows % 2 == 0) else 1
    rpg = rows // G
    x = torch.randn(rows, cols, device=DEV, dtype=dtype, requires_grad=True)
    res = torch.randn(rows, cols, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(cols, device=DEV)).requires_grad_(True)
    b = (0.1 * torch.randn(cols, device=DEV)).requires_grad_(True)
    gam = torch.randn(G, cols, device=DEV, requires_grad=True) if film else None
    bet = torch.randn(G, cols, device=DEV, requires_grad=True) if film else None
    y, xs = ops.layer_norm(x, w, b, 1e-5, res=res, gamma=gam, beta=bet, rows_per_group=rpg)
    gy = torch.randn_like(y)
    gs = torch.randn_like(xs)
    (y.float() * gy.float()).sum().add((xs.float() * gs.float()).sum()).backward()
    # fp64 reference
    X, Rr, W, Bb = (t.detach().double().requires_grad_(True) for t in (x, res, w, b))
    S = X + Rr
    Y = R.layer_norm_ref(S, W, Bb)
    if film:
        Gm, Bt = (t.detach().double().requires_grad_(True) for t in (gam, bet))
        Y = (Gm.repeat_interleave(rpg, 0) * Y + Bt.repeat_interleave(rpg, 0))
    (Y * gy.double()).sum().add((S * gs.double()).sum()).backward()
    tol = 1e-3 if dtype == torch.float32 else 2e-2
    close(y.float(), Y.detach(), rtol=tol, name="y")
    close(x.grad.float(), X.grad, rtol=tol, name="dx")
    close(res.grad.float(), Rr.grad, rtol=tol, name="dres")
    close(w.grad, W.grad, rtol=tol, name="dw")
    close(b.grad, Bb.grad, rtol=tol, name="db")
    if film:
        close(gam.grad, Gm.grad, rtol=tol, name="dgamma")
        close(bet.grad, Bt.grad, rtol=tol, name="dbeta")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols,rows", [(1024, 128), (512, 100), (64, 7)])
def test_layernorm_film_tensor_and_dx_colsum(dtype, cols, rows):
    """ONE (G, 2N) gamma | beta FiLM tensor (gradient written in place, side by
    side) equals separate gamma / beta; the backward's fused column sums of dx
    (colsum_slot, the upstream linear's bias gradient) equal the column sums of
    the dx it stores, as stored (dtype-rounded), in fp32."""
    from mtts import ops
    from mtts.linear import BiasGradSlot, colsum
    torch.manual_seed(cols + rows)
    G = 2 if rows % 2 == 0 else 1
    rpg = rows // G
    x = torch.randn(rows, cols, device=DEV, dtype=dtype)
    res = torch.randn(rows, cols, device=DEV, dtype=dtype)
    w = 1 + 0.1 * torch.randn(cols, device=DEV)
    b = 0.1 * torch.randn(cols, device=DEV)
    gb = torch.randn(G, 2 * cols, device=DEV)
    gy = torch.randn(rows, cols, device=DEV, dtype=dtype)
    gs = torch.randn(rows, cols, device=DEV, dtype=dtype)
    outs = []
    for mode in ("split", "tensor"):
        xx, rr = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
        if mode == "split":
            gam = gb[:, :cols].clone().requires_grad_(True)
            bet = gb[:, cols:].clone().requires_grad_(True)
            slot = None
            y, xs = ops.layer_norm(xx, w, b, 1e-5, res=rr, gamma=gam, beta=bet, rows_per_group=rpg)
        else:
            film = gb.clone().requires_grad_(True)
            slot = BiasGradSlot()
            y, xs = ops.layer_norm(xx, w, b, 1e-5, res=rr, rows_per_group=rpg, film=film, colsum_slot=slot)
        (y.float() * gy.float()).sum().add((xs.float() * gs.float()).sum()).backward()
        dfilm = torch.cat([gam.grad, bet.grad], 1) if mode == "split" else film.grad
        outs.append((y, xx.grad, rr.grad, dfilm, slot))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])
    assert outs[1][3].shape == (G, 2 * cols) and torch.equal(outs[0][3], outs[1][3])
    cs = outs[1][4].take(cols)
    assert cs is not None and cs.dtype == torch.float32
    close(cs, colsum(outs[1][1]), rtol=1e-5, name="dx column sums")


def test_upstream_signature_ops(golden):
    """mamba-ssm-signature wrappers ((B, D, L) layout) incl. autograd."""
    from mtts import ops
    g = golden("scan_full.npz")
    ins = {k: torch.from_numpy(g[k]).to(DEV).requires_grad_(True) for k in
           ("u", "delta", "A", "B", "C", "D", "z", "delta_bias")}
    out = ops.selective_scan_fn(ins["u"], ins["delta"], ins["A"], ins["B"], ins["C"], ins["D"], ins["z"],
                                ins["delta_bias"], delta_softplus=True)
    close(out, g["out"], name="out")
    (out * torch.from_numpy(g["dout"]).to(DEV)).sum().backward()
    for k, t in ins.items():
        close(t.grad, g["d" + k], name="d" + k)


@pytest.mark.parametrize("rows,cols", [(1, 5), (300, 64), (16384, 1024), (4097, 96), (20000, 2050), (1024, 1024), (256, 512), (777, 384)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_colsum(rows, cols, dtype):
    from mtts.linear import colsum
    torch.manual_seed(rows)
    x = torch.randn(rows, cols, device=DEV).to(dtype)
    close(colsum(x), x.double().sum(0), rtol=1e-5, name="colsum")
    if rows > 1:
        close(colsum(x[:, 1:]), x[:, 1:].double().sum(0), rtol=1e-5, name="colsum strided")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rpg,groups", [(1090, 3), (2048, 2), (700, 4), (1300, 1)])
def test_colsum_groups_ragged(dtype, rpg, groups):
    """Per-group column sums (mtts_colsum rows_per_group): groups of > 1024
    rows that are not a multiple of 256 (the style frames' per-batch sums)
    end in a ragged chunk; every group sums exactly its own rows."""
    from mtts.linear import colsum_groups
    torch.manual_seed(rpg)
    x = torch.randn(rpg * groups, 320, device=DEV).to(dtype)
    close(colsum_groups(x, rpg), x.double().view(groups, rpg, -1).sum(1), rtol=1e-5, name="colsum_groups")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_fn_grads(dtype):
    from mtts.linear import linear
    torch.manual_seed(0)
    x = torch.randn(4, 1024, 96, device=DEV).to(dtype).requires_grad_(True)
    w = torch.randn(160, 96, device=DEV, requires_grad=True)
    b = torch.randn(160, device=DEV, requires_grad=True)
    y = linear(x, w, b, rows=(32, 128))
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr, wr, br = x.detach().double().requires_grad_(True), w.detach().double().requires_grad_(True), \
        b.detach().double().requires_grad_(True)
    yr = xr @ wr[32:128].t() + br[32:128]
    (yr * g.double()).sum().backward()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    close(y.float(), yr, rtol=tol, name="y")
    close(x.grad.float(), xr.grad, rtol=tol, name="dx")
    close(w.grad, wr.grad, rtol=tol, name="dw")
    close(b.grad, br.grad, rtol=tol, name="db")


@pytest.mark.parametrize("shapes", [[(4096, 1024), (10, 1024), (96, 2048), (3000,), (2048, 64), (1024, 1024)],
                                    [(130, 70), (64, 64), (5,), (513, 520)]])
def test_cast_bf16_multi(shapes):
    """mtts_cast_bf16_multi (one launch over a parameter list) == torch's RNE
    .to(bfloat16) and its transpose, exact, for full / ragged tiles and 1-D."""
    from mtts import _lib as L
    from mtts.linear import _cast_multi_bf16, _want_t, TRANSPOSE_MIN
    torch.manual_seed(0)
    ps = [torch.randn(*s, device=DEV) * 3 for s in shapes]
    _cast_multi_bf16(ps)
    for p in ps:
        ref = p.to(torch.bfloat16)
        assert torch.equal(p._mtts_cast[1], ref)
        if _want_t(p):
            assert torch.equal(p._mtts_castT[1], ref.t().contiguous())
        elif p.dim() == 2 and min(p.shape) < TRANSPOSE_MIN:
            assert getattr(p, "_mtts_castT", None) is None
    ps[0].add_(1.0)                # a later step re-casts the same buffers in place
    _cast_multi_bf16(ps)
    assert torch.equal(ps[0]._mtts_cast[1], ps[0].to(torch.bfloat16))


@pytest.mark.parametrize("M,N,K,bias,act", [(32, 4096, 1024, False, None), (32, 96, 2048, False, None),
                                            (32, 2048, 64, False, None), (32, 1024, 2048, True, None),
                                            (32, 2048, 1024, True, "gelu"), (32, 10, 1024, True, None),
                                            (7, 130, 192, True, "gelu"), (1, 33, 64, False, None)])
def test_gemm_rows(M, N, K, bias, act):
    """Decode-step skinny GEMM (csrc/rows.hip) vs a float64 reference of the
    same bf16 operands; bound: one bf16 rounding of the output (2^-8 relative
    to max|y|)."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16) if bias else None
    y = ops.gemm_rows(x, w, b, act)
    ref = x.double() @ w.double().t()
    if b is not None:
        ref = ref + b.double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    close(y, ref, rtol=2 ** -8, name="gemm_rows")
    # strided x view (x_dbl[:, :dt_rank] in the decode step)
    xb = torch.randn(M, K + 64, generator=g).to(DEV, torch.bfloat16)
    close(ops.gemm_rows(xb[:, :K], w), xb[:, :K].double() @ w.double().t(), rtol=2 ** -8, name="strided")


@pytest.mark.parametrize("dtype,R", [(torch.float32, 64), (torch.bfloat16, 64), (torch.bfloat16, 4),
                                     (torch.float32, 7)])
def test_state_update_fused_dt_proj(dtype, R):
    """dt_proj fused into the state update (dt_rank > 0, strided B / C views of
    x_dbl) equals dt_proj as a separate fp32 product followed by the plain
    update, within one bf16 rounding of delta for bf16 I/O."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(R)
    Bsz, D, N = 5, 96, 16
    x_dbl = torch.randn(Bsz, R + 2 * N, generator=g).to(DEV, dtype)
    u = torch.randn(Bsz, D, generator=g).to(DEV, dtype)
    z = torch.randn(Bsz, D, generator=g).to(DEV, dtype)
    w = (torch.randn(D, R, generator=g) / R ** 0.5).to(DEV, dtype)
    A = -torch.rand(D, N, generator=g).to(DEV) - 0.5
    Dv = torch.randn(D, generator=g).to(DEV)
    bias = torch.randn(D, generator=g).to(DEV) * 0.1
    st0 = torch.randn(Bsz, D, N, generator=g).to(DEV)
    s1, s2 = st0.clone(), st0.clone()
    y1 = ops.state_update(s1, u, x_dbl[:, :R], A, x_dbl[:, R:R + N], x_dbl[:, R + N:], Dv, z, bias, True, dt_w=w)
    delta = (x_dbl[:, :R].float() @ w.float().t()).to(dtype)
    y2 = ops.state_update(s2, u, delta, A, x_dbl[:, R:R + N].contiguous(), x_dbl[:, R + N:].contiguous(), Dv, z,
                          bias, True)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    close(s1, s2, rtol=tol, name="state")
    close(y1.float(), y2.float(), rtol=tol, name="y")


@pytest.mark.parametrize("M,C,N", [(32, 2048, 4096), (3, 128, 256)])
def test_gemm_rows_conv_epilogue(M, C, N):
    """in_proj with the causal-conv1d update + SiLU folded into its epilogue
    equals in_proj followed by mtts_causal_conv1d_update (state and u)."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(C)
    K = 128
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    cw, cb = torch.randn(C, 4, generator=g).to(DEV), torch.randn(C, generator=g).to(DEV)
    st = torch.randn(M, C, 4, generator=g).to(DEV)
    st2 = st.clone()
    for _ in range(2):
        y, u = ops.gemm_rows(x, w, conv=(st, cw, cb))
        y2 = ops.gemm_rows(x, w)
        u2 = ops.conv_update(y2[:, :C], st2, cw, cb, True)
        assert torch.equal(y, y2)
        close(st, st2, rtol=1e-6, name="conv state")
        close(u.float(), u2.float(), rtol=2 ** -8, name="u")


@pytest.mark.parametrize("M,N,K", [(32, 4096, 1024), (32, 1024, 256), (5, 512, 512), (7, 96, 128), (3, 64, 64)])
@pytest.mark.parametrize("film", [False, True])
def test_gemm_rows_ln_prologue_and_residual(M, N, K, film):
    """LayerNorm (+FiLM) prologue of the decode projections (statistics from
    the operand registers) against mtts_layernorm_fwd followed by the plain
    GEMM: the same arithmetic up to fp32 summation order of mean / variance,
    so within one bf16 rounding of the normalised operand; the residual
    epilogue equals the LayerNorm kernel's x_sum bit for bit."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(M * N + K)
    x = (torch.randn(M, K, generator=g) * 3 + 0.5).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    lw, lb = torch.randn(K, generator=g).to(DEV), torch.randn(K, generator=g).to(DEV)
    gam = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    bet = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    y = ops.gemm_rows(x, w, b, ln=(lw, lb, 1e-5, gam, bet))
    h, _ = ops.layer_norm(x, lw, lb, 1e-5, gamma=gam, beta=bet, rows_per_group=1)
    y2 = ops.gemm_rows(h, w, b)
    close(y.float(), y2.float(), rtol=2 ** -7, name="ln prologue")
    assert (y != y2).float().mean().item() < 0.02      # bf16-level disagreements are rare
    res = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    xs = ops.gemm_rows(x, w, b, res=res)
    if N % 512 == 0:
        _, xs2 = ops.layer_norm(ops.gemm_rows(x, w, b), torch.ones(N, device=DEV), torch.zeros(N, device=DEV),
                                1e-5, res=res)
        assert torch.equal(xs, xs2)
    close(xs.float(), ops.gemm_rows(x, w, b).float() + res.float(), rtol=2 ** -7, name="residual")


def test_gemm_rows_ln_prologue_rejects_multi_trip_k(monkeypatch):
    """One workgroup per tile: the LayerNorm prologue needs one trip per wave
    (K = 4096 cannot); split over workgroups the same K is taken."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.randn(4, 4096, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(64, 4096, generator=g) / 64).to(DEV, torch.bfloat16)
    lw, lb = torch.ones(4096, device=DEV), torch.zeros(4096, device=DEV)
    monkeypatch.setattr(ops, "ROWS_SPLITK", False)
    with pytest.raises(RuntimeError, match="LayerNorm prologue"):
        ops.gemm_rows(x, w, ln=(lw, lb, 1e-5))
    monkeypatch.setattr(ops, "ROWS_SPLITK", True)
    with pytest.raises(RuntimeError, match="LayerNorm prologue"):   # 4096 > 2048: LDS copy of the LN params
        ops.gemm_rows(x, w, ln=(lw, lb, 1e-5))
    x2, w2, lw2, lb2 = x[:, :2048], w[:, :2048].contiguous(), lw[:2048], lb[:2048]
    y = ops.gemm_rows(x2, w2, ln=(lw2, lb2, 1e-5))
    h, _ = ops.layer_norm(x2.contiguous(), lw2, lb2, 1e-5, rows_per_group=1)
    close(y.float(), (h.double() @ w2.double().t()).float(), rtol=2 ** -7, name="split-K LN K=2048")


@pytest.mark.parametrize("M,N,K", [(32, 4096, 1024), (32, 1024, 2048), (32, 1024, 1024), (32, 96, 2048),
                                   (32, 10, 1024), (5, 2048, 1024), (3, 800, 512)])
@pytest.mark.parametrize("mode", ["plain", "ln", "film", "res", "conv", "gelu"])
def test_gemm_rows_split_k_matches_single_workgroup(M, N, K, mode, monkeypatch):
    """The K range split over workgroups (fp32 partial slabs, last arriver
    sums them in fixed order) equals one workgroup per tile up to fp32
    summation order: within one bf16 rounding, and bit-identical across
    repeated launches (deterministic); tickets left at zero."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K + len(mode))
    x = (torch.randn(M, K, generator=g) * 2 + 0.3).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    kw = {}
    if mode in ("ln", "film"):
        if not ops.gemm_rows_ln_ok(K):
            pytest.skip("K not a single-workgroup LayerNorm size")
        lw, lb = torch.randn(K, generator=g).to(DEV), torch.randn(K, generator=g).to(DEV)
        gam = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if mode == "film" else None
        bet = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if mode == "film" else None
        kw["ln"] = (lw, lb, 1e-5, gam, bet)
    if mode == "res":
        kw["res"] = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    act = "gelu" if mode == "gelu" else None
    C = (N // 2) // 32 * 32
    if mode == "conv" and C == 0:
        pytest.skip("no whole conv tile")
    st0 = torch.randn(M, C, 4, generator=g).to(DEV) if mode == "conv" else None
    outs = []
    for split in (False, True, True):
        monkeypatch.setattr(ops, "ROWS_SPLITK", split)
        if mode == "conv":
            st = st0.clone()
            y, u = ops.gemm_rows(x, w, conv=(st, torch.ones(C, 4, device=DEV), None))
            outs.append((y, u, st))
        else:
            outs.append((ops.gemm_rows(x, w, b, act, **kw),))
    for a, c in zip(outs[0], outs[1]):
        close(c.float(), a.float(), rtol=2 ** -7, name=f"split-K {mode}")
    for a, c in zip(outs[1], outs[2]):
        assert torch.equal(a, c)
    if ops.rows_kgroups(N, K, "ln" in kw) > 1:
        assert int(ops.rows_workspace(DEV)[1].abs().sum()) == 0


def test_wgrad_split_k_matches_fp64():
    from mtts.linear import wgrad
    g = torch.Generator(device="cpu").manual_seed(5)
    dy = torch.randn(8192, 1024, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(8192, 2048, generator=g).to(DEV, torch.bfloat16)
    ref = dy.double().t() @ x.double()
    close(wgrad(dy, x), ref, rtol=1e-5, name="wgrad")
    big = torch.zeros(3072, 2048, device=DEV)
    wgrad(dy, x, out=big[1024:2048])
    close(big[1024:2048], ref, rtol=1e-5, name="wgrad row slice")
    assert big[:1024].abs().max().item() == 0 and big[2048:].abs().max().item() == 0


@pytest.mark.parametrize("M", [8720, 1089])
def test_wgrad_ragged_token_count(M):
    """A token count that is not a multiple of 64 (the style frames): the
    aligned bulk on the TN kernel plus the < 64 remainder rows, into a fresh
    tensor and into a row slice of a larger one."""
    from mtts.linear import wgrad
    g = torch.Generator(device="cpu").manual_seed(M)
    dy = torch.randn(M, 1024, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(M, 512, generator=g).to(DEV, torch.bfloat16)
    ref = dy.double().t() @ x.double()
    close(wgrad(dy, x), ref, rtol=1e-5, name="wgrad ragged")
    big = torch.zeros(2048, 512, device=DEV)
    wgrad(dy, x, out=big[512:1536])
    close(big[512:1536], ref, rtol=1e-5, name="wgrad ragged row slice")
    assert big[:512].abs().max().item() == 0 and big[1536:].abs().max().item() == 0


@pytest.mark.parametrize("M,N,K", [(32, 4096, 1024), (32, 1024, 2048), (32, 1024, 4096), (32, 96, 2048),
                                   (32, 10, 1024), (5, 2048, 1024), (3, 800, 512), (17, 64, 64), (16, 48, 192)])
@pytest.mark.parametrize("mode", ["plain", "ln", "film", "res", "conv", "gelu"])
def test_gemm_rows_packed_matches_row_major(M, N, K, mode):
    """Packed decode weights (mtts_pack_rows_weight + csrc/gemv.hip: 16-column
    tiles, coalesced KiB weight loads, K over up to 8 waves) equal the
    row-major skinny GEMM up to fp32 summation order (one bf16 rounding,
    bound 2^-7 relative), bit-identical across repeated launches; the packed
    image holds exactly the weight's fragments (zero-padded columns)."""
    from mtts import ops
    if not ops.gemv_split_ok(K, ln=mode in ("ln", "film")):
        pytest.skip("K not taken by the packed kernel")
    g = torch.Generator(device="cpu").manual_seed(M * 3 + N + K + len(mode))
    x = (torch.randn(M, K, generator=g) * 2 + 0.3).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    wp = ops.pack_rows_weight(w)
    # the image: tile t, step s, lane l holds W[16t + l%16, 32s + 8(l/16) : +8]
    Np = -(-N // 16) * 16
    wpad = torch.zeros(Np, K, device=DEV, dtype=torch.bfloat16)
    wpad[:N] = w
    img = wpad.view(Np // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1)
    assert torch.equal(wp.data, img)
    kw, act = {}, None
    if mode in ("ln", "film"):
        lw, lb = torch.randn(K, generator=g).to(DEV), torch.randn(K, generator=g).to(DEV)
        gam = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if mode == "film" else None
        bet = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if mode == "film" else None
        kw["ln"] = (lw, lb, 1e-5, gam, bet)
    if mode == "res":
        kw["res"] = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    if mode == "gelu":
        act = "gelu"
    C = (N // 2) // 32 * 32
    if mode == "conv":
        if C == 0:
            pytest.skip("no whole conv tile")
        st0 = torch.randn(M, C, 4, generator=g).to(DEV)
        cw, cb = torch.randn(C, 4, generator=g).to(DEV), torch.randn(C, generator=g).to(DEV)
        outs = []
        for wt in (w, wp, wp):
            st = st0.clone()
            y, u = ops.gemm_rows(x, wt, conv=(st, cw, cb))
            outs.append((y, u, st))
    elif "ln" in kw and not ops.gemm_rows_ln_ok(K):   # row-major prologue cannot: LayerNorm kernel + GEMM
        h, _ = ops.layer_norm(x, kw["ln"][0], kw["ln"][1], 1e-5, gamma=kw["ln"][3], beta=kw["ln"][4],
                              rows_per_group=1)
        outs = [(ops.gemm_rows(h, w, b),)] + [(ops.gemm_rows(x, wp, b, **kw),) for _ in range(2)]
    else:
        outs = [(ops.gemm_rows(x, wt, b, act, **kw),) for wt in (w, wp, wp)]
    for a_, c_ in zip(outs[0], outs[1]):
        close(c_.float(), a_.float(), rtol=2 ** -7, name=f"packed {mode}")
    for a_, c_ in zip(outs[1], outs[2]):
        assert torch.equal(a_, c_)
    if mode == "plain":
        ref = x.double() @ w.double().t() + b.double()
        close(outs[1][0], ref, rtol=2 ** -8, name="packed vs float64")


@pytest.mark.parametrize("M,K", [(32, 1024), (5, 256), (17, 2048)])
@pytest.mark.parametrize("film", [False, True])
def test_ln_rows_packed_equals_layer_norm(M, K, film):
    """mtts_layernorm_rows_packed: the packed image of LN(+FiLM) equals
    mtts_layernorm_fwd's y bit for bit (same arithmetic and order)."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(M + K + film)
    x = (torch.randn(M, K, generator=g) * 3 + 0.5).to(DEV, torch.bfloat16)
    lw, lb = torch.randn(K, generator=g).to(DEV), torch.randn(K, generator=g).to(DEV)
    gam = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    bet = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    hp = ops.ln_rows_packed(x, lw, lb, 1e-5, gam, bet)
    h, _ = ops.layer_norm(x, lw, lb, 1e-5, gamma=gam, beta=bet, rows_per_group=1)
    assert torch.equal(hp.unpack(), h)


@pytest.mark.parametrize("M,N,K", [(32, 1024, 2048), (32, 4096, 1024), (7, 96, 512), (20, 64, 64)])
def test_gemm_rows_packed_activations(M, N, K):
    """Packed activation images (csrc/common.h xpk_index) in and out of the
    packed projection kernel: x as an image gives the row-major result bit
    for bit; the y / u images unpack to the row-major y / u; state update and
    decode attention images unpack to their row-major outputs."""
    from mtts import ops
    from mtts.attn_kernels import attention_decode_packed, attention_fwd
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    wp = ops.pack_rows_weight(w)
    xp = ops.PackedAct.empty(M, K, DEV)
    xp.data.view(-1)[:] = 0
    # build the image through a producer: y of an identity-free GEMM is awkward, so scatter directly
    img = torch.zeros(32, K, device=DEV, dtype=torch.bfloat16)
    img[:M] = x
    xp.data.copy_(img.view(2, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).reshape(-1))
    assert torch.equal(xp.unpack(), x)
    y_ref = ops.gemm_rows(x, wp, b, res=None)
    y2, yp = ops.gemm_rows(xp, wp, b, packed_out="also")
    assert torch.equal(y2, y_ref)
    assert torch.equal(yp.unpack(), y_ref)
    yo = ops.gemm_rows(xp, wp, b, "gelu", packed_out="only")
    assert torch.equal(yo.unpack(), ops.gemm_rows(x, wp, b, "gelu"))
    if N % 64 == 0:   # conv epilogue with a packed u
        C = N // 2
        st0 = torch.randn(M, C, 4, generator=g).to(DEV)
        cw, cb = torch.randn(C, 4, generator=g).to(DEV), torch.randn(C, generator=g).to(DEV)
        s1, s2 = st0.clone(), st0.clone()
        ya, ua = ops.gemm_rows(xp, wp, conv=(s1, cw, cb))
        yb, ub, upk = ops.gemm_rows(x, wp, conv=(s2, cw, cb), u_packed=True)
        assert torch.equal(ya, yb) and torch.equal(ua, ub) and torch.equal(s1, s2)
        assert torch.equal(upk.unpack(), ub)
    if K % 32 == 0 and M <= 32:   # state update image
        D, Nst = K, 16
        st = torch.randn(M, D, Nst, generator=g).to(DEV)
        u = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
        z = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
        dt = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
        Bm = torch.randn(M, Nst, generator=g).to(DEV, torch.bfloat16)
        Cm = torch.randn(M, Nst, generator=g).to(DEV, torch.bfloat16)
        A = -torch.rand(D, Nst, generator=g).to(DEV) - 0.5
        Dv = torch.randn(D, generator=g).to(DEV)
        s1, s2 = st.clone(), st.clone()
        y1 = ops.state_update(s1, u, dt, A, Bm, Cm, Dv, z, None, True)
        y2p = ops.state_update(s2, u, dt, A, Bm, Cm, Dv, z, None, True, packed_out=True)
        assert torch.equal(s1, s2) and torch.equal(y2p.unpack(), y1)
    if K in (512, 1024, 2048):   # decode attention image
        H = K // 128 if K >= 1024 else K // 64
        q = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        kv = torch.randn(M, 77, 2 * K, generator=g).to(DEV, torch.bfloat16)
        kpm = torch.zeros(M, 77, dtype=torch.bool, device=DEV)
        kpm[:, 70:] = True
        o, _ = attention_fwd(q[:, None], kv[..., :K], kv[..., K:], H, kpm)
        op = attention_decode_packed(q, kv[..., :K], kv[..., K:], H, kpm)
        assert torch.equal(op.unpack(), o[:, 0])


@pytest.mark.parametrize("M,N,K", [(32, 4096, 1024), (9, 1024, 512)])
@pytest.mark.parametrize("film", [False, True])
def test_gemm_rows_ln_prologue_on_packed_x(M, N, K, film):
    """LayerNorm(+FiLM) prologue on a packed x (FiLM rows packed too) equals
    the same prologue on the row-major x bit for bit (same registers, same
    order), and the residual epilogue's packed copy of y unpacks to y."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K + film)
    x = (torch.randn(M, K, generator=g) * 2 + 0.3).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    lw, lb = torch.randn(K, generator=g).to(DEV), torch.randn(K, generator=g).to(DEV)
    gam = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    bet = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if film else None
    wp = ops.pack_rows_weight(w)
    y1 = ops.gemm_rows(x, wp, b, ln=(lw, lb, 1e-5, gam, bet))
    xp = ops.PackedAct.pack(x)
    gp = ops.PackedAct.pack(gam) if film else None
    bp = ops.PackedAct.pack(bet) if film else None
    y2 = ops.gemm_rows(xp, wp, b, ln=(lw, lb, 1e-5, gp, bp))
    assert torch.equal(y1, y2)
    res = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    y3, y3p = ops.gemm_rows(xp, wp, b, res=res, packed_out="also")
    assert torch.equal(y3p.unpack(), y3)
    assert torch.equal(y3, ops.gemm_rows(x, wp, b, res=res))


@pytest.mark.parametrize("M,N,K", [(1, 4096, 64), (3, 2048, 64)])
def test_gemm_rows_packed_no_bias_wide_n_small_k(M, N, K):
    """Packed projection without bias / residual where N far exceeds the x
    operand's size (the absent operands' dummy loads must stay inside an
    allocation): equals the float64 product within one bf16 rounding."""
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    y = ops.gemm_rows(x, ops.pack_rows_weight(w))
    close(y, x.double() @ w.double().t(), rtol=2 ** -8, name="packed no-bias")
    yp = ops.gemm_rows(ops.PackedAct.pack(x), ops.pack_rows_weight(w), packed_out="only")
    assert torch.equal(yp.unpack(), y)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 100, 256), (1, 37, 100), (32, 48, 2048), (2, 300, 128)])
def test_scan_a_is_log_matches_explicit_A(shape, dtype):
    """a_is_log (A = -exp(A_log) formed in-kernel, the backward returning
    dA_log = dA * A) equals passing the explicit A: every kernel family
    (one-lane-per-channel at B*D >= 64k, LDS-DMA P = 4, narrow D, L-segment
    backward)."""
    from mtts import ops
    torch.manual_seed(5)
    B, L, D = shape
    u = torch.randn(B, L, D, device=DEV).to(dtype)
    delta = (torch.randn(B, L, D, device=DEV) * 0.5).to(dtype)
    z = torch.randn(B, L, D, device=DEV).to(dtype)
    Bm = torch.randn(B, L, 16, device=DEV).to(dtype)
    Cm = torch.randn(B, L, 16, device=DEV).to(dtype)
    A_log = torch.log(torch.arange(1, 17, device=DEV, dtype=torch.float32)).repeat(D, 1) + 0.1 * torch.randn(D, 16, device=DEV)
    A = -torch.exp(A_log)
    Dp = torch.randn(D, device=DEV)
    bias = torch.randn(D, device=DEV) * 0.1
    y1, _, ck1 = ops.scan_fwd(u, delta, A, Bm, Cm, Dp, z, bias, True, want_ckpt=True)
    y2, _, ck2 = ops.scan_fwd(u, delta, A_log, Bm, Cm, Dp, z, bias, True, want_ckpt=True, a_is_log=True)
    close(y2.float(), y1.float(), rtol=1e-5 if dtype == torch.float32 else 1e-2, name="out")
    g = torch.randn(B, L, D, device=DEV).to(dtype)
    r1 = ops.scan_bwd(u, delta, A, Bm, Cm, Dp, z, bias, True, None, ck1, g)
    r2 = ops.scan_bwd(u, delta, A_log, Bm, Cm, Dp, z, bias, True, None, ck2, g, a_is_log=True)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for name, i in (("du", 0), ("ddelta", 1), ("dz", 2), ("dB", 3), ("dC", 4), ("dD", 6), ("dbias", 7)):
        close(r2[i].float(), r1[i].float(), rtol=tol, name=name)
    close(r2[5], r1[5] * A, rtol=tol, name="dA_log")


