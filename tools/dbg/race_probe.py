"""Bitwise determinism of the training-step kernels under GPU sharing: NPROC
processes run the same probe on cuda:0 at once; each op is run REPS times on
fixed inputs and compared bit for bit with its first result.  A kernel with an
intra-workgroup race (LDS read before its write is visible, a missing wait)
shows up as mismatches when other work shares its CUs.
  NPROC=2 python tools/dbg/race_probe.py
BG=1 ONLY0=<probe> ONLY1=<other probes>: process 1 runs its probes back to back
(unchecked) for as long as process 0 checks its own."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

REPS = int(os.environ.get("REPS", "30"))


def probes(dev):
    from mtts import attn_kernels as AK
    from mtts import gemm as G
    from mtts import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    bf = torch.bfloat16
    r = lambda *s, sc=1.0, dt=bf: (torch.randn(*s, generator=g) * sc).to(dev, dt)  # noqa: E731
    out = {}
    for (B, T, S, d, H) in [(2, 512, 64, 256, 4), (8, 2048, 128, 1024, 8)]:
        q, kv, dout = r(B, T, d), r(B, S, 2 * d), r(B, T, d)
        kpm = torch.zeros(B, S, dtype=torch.bool, device=dev)
        kpm[0, S - 14:] = True
        o, lse = AK.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)

        def attn(q=q, kv=kv, o=o, lse=lse, dout=dout, kpm=kpm, H=H, d=d):
            dkv = torch.empty_like(kv)
            dq, _, _ = AK.attention_bwd(q, kv[..., :d], kv[..., d:], H, kpm, o, lse, dout, dk=dkv[..., :d],
                                        dv=dkv[..., d:])
            o2, _ = AK.attention_fwd(q, kv[..., :d], kv[..., d:], H, kpm, want_lse=True)
            return [dq, dkv, o2]
        out[f"attn B{B} T{T} S{S} d{d}"] = attn
        x, res, dy = r(B * T, d), r(B * T, d), r(B * T, d)
        w, b = torch.randn(d, device=dev), torch.randn(d, device=dev)
        gb = torch.randn(B, 2 * d, device=dev)

        def ln(x=x, res=res, dy=dy, w=w, b=b, gb=gb, T=T, d=d):
            xx = x.clone().requires_grad_(True)
            film = gb.clone().requires_grad_(True)
            from mtts.linear import BiasGradSlot
            slot = BiasGradSlot()
            y, xs = ops.layer_norm(xx, w, b, 1e-5, res=res, rows_per_group=T, film=film, colsum_slot=slot)
            (y.float() * dy.float()).sum().backward()
            return [y, xs, xx.grad, film.grad, slot.value]
        out[f"ln+film d{d}"] = ln
    # scan / conv at C2 shape (SCAN_SHAPE=B,L,D: another shape, e.g. the DP
    # test's 2,512,512)
    B, L, D = (int(v) for v in os.environ.get("SCAN_SHAPE", "8,2048,2048").split(","))
    u, dl, z, dy = r(B, L, D), r(B, L, D, sc=0.3), r(B, L, D), r(B, L, D)
    A = -torch.rand(D, 16, device=dev) - 0.1
    Bm, Cm = r(B, L, 16), r(B, L, 16)
    Dp, bias = torch.randn(D, device=dev), torch.randn(D, device=dev) * 0.1

    y0, last0, ck0 = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True, want_ckpt=True)

    def scan_fwd():
        y, last, ck = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, z, bias, True, want_last=True, want_ckpt=True)
        return [y, last, ck]
    out["scan fwd C2 (y, last, ckpt)"] = scan_fwd

    from mtts import _lib

    def scan_bwd(segs=None):
        with _lib.override(scan_bwd_segs=segs):
            gr = ops.scan_bwd(u, dl, A, Bm, Cm, Dp, z, bias, True, None, ck0, dy)
        return [t for t in gr if t is not None]
    out["scan bwd C2 (du, ddelta, dz, dB, dC, dA, dD, dbias)"] = scan_bwd
    out["scan bwd C2 one segment (no carry kernel)"] = lambda: scan_bwd(1)
    from mtts import _lib as LL
    nws = LL.lib().mtts_selective_scan_bwd_workspace(B, D, L, 16)
    nblk = D // 64
    nslab = B * nblk * L * 32

    K6 = ((nws - 256) // 4 - B * nblk * L * 32) // (B * D * 35)   # segments of the backward's plan

    def scan_bwd_ws(u, dl, Bm, Cm, z, ck, dy):
        # workspace poisoned with NaN (0xFF bytes): an entry the kernels did not
        # write this call stays NaN (bitwise compare: equal when unwritten in
        # both runs); the call's du, ddelta, dB and reduced dA / dD / dbias too
        ws = torch.full((nws,), 255, device=dev, dtype=torch.uint8)
        gr = ops.scan_bwd(u, dl, A, Bm, Cm, Dp, z, bias, True, None, ck, dy, workspace=ws)
        f = ws[:(nws // 4) * 4].view(torch.float32)
        npar = B * K6 * D * 18
        return [f[:nslab], f[nslab:nslab + npar], f[nslab + npar:nslab + npar + B * K6 * D * 17], gr[0], gr[1],
                gr[3]] + [t for t in gr[5:8] if t is not None]
    out["scan bwd C2 workspace (slab, par, seg, du, ddelta, dB, dA, dD, dbias)"] = \
        lambda: scan_bwd_ws(u, dl, Bm, Cm, z, ck0, dy)
    u32, dl32, z32, dy32 = (t.float() for t in (u, dl, z, dy))
    ck32 = ops.scan_fwd(u32, dl32, A, Bm.float(), Cm.float(), Dp, z32, bias, True, want_ckpt=True)[2]
    out["scan bwd C2 fp32"] = lambda: [t for t in ops.scan_bwd(u32, dl32, A, Bm.float(), Cm.float(), Dp, z32, bias, True,
                                                                None, ck32, dy32) if t is not None]
    out["scan bwd C2 fp32 workspace (slab, par, seg, du, ddelta, dB, dA, dD, dbias)"] = \
        lambda: scan_bwd_ws(u32, dl32, Bm.float(), Cm.float(), z32, ck32, dy32)
    r_ = 32 if D >= 1024 else 16
    dd2, dt2 = r(B * L, D), r(B * L, r_)
    gx, u2 = r(B * L, r_ + 32), r(B * L, D)
    out["skinny tn (dW_dt, dW_x)"] = lambda: [G.mm_skinny_tn(dd2, dt2), G.mm_skinny_tn(u2, gx, trans_c=True)]
    xz = r(B, L, 2 * D)
    cw, cb = torch.randn(D, 4, device=dev) * 0.5, torch.randn(D, device=dev) * 0.1

    def conv():
        o, _ = ops.conv_fwd(xz[..., :D], cw, cb, True)
        dxz = torch.zeros_like(xz)
        _, dw, db = ops.conv_bwd(xz[..., :D], cw, cb, dy, True, dx=dxz[..., :D])
        return [o, dxz, dw, db]
    out["conv C2"] = conv
    a1, w1 = r(16384, 1024), r(4096, 1024)
    dyy, xx = r(16384, 4096), r(16384, 1024)

    def gemm():
        return [G.mm_nt(a1, w1), G.mm_tn(dyy, xx)]
    out["gemm nt/tn"] = gemm
    gb1 = torch.randn(4096, device=dev)
    pre1 = r(16384, 4096)

    def gemm_gelu():
        # the FFN epilogues: bias + GELU (packed-f32 polynomial beside the
        # tile's MFMA waves) writing the pre-activation, and GELU backward
        aux = torch.empty(16384, 4096, device=dev, dtype=bf)
        y = G.mm_nt(a1, w1, bias=gb1, gelu_aux=aux)
        return [y, aux, G.mm_nt(a1, w1, dgelu_aux=pre1)]
    out["gemm gelu / dgelu epilogues"] = gemm_gelu
    # round-6 kernels: dropout forms, the codec token-table gradient, ragged
    # per-group column sums, the grouped TN weight-gradient launch
    from mtts import dropout as DO
    from mtts import wgrad as WG
    from mtts.embed import _table_grad
    from mtts.linear import colsum_groups
    xd, v8 = r(8 * 1090, 1024), r(8, 1024)
    dpre, pre = r(8 * 1090, 4096), r(8 * 1090, 4096)
    out["dropout (plain, group, broadcast, dgelu)"] = lambda: [
        DO.apply_mask(xd, 0.1, 77), DO.apply_mask(xd, 0.1, 77, group=128),
        DO.apply_mask(v8, 0.1, 77, group=128, rep=1090), DO.apply_mask(dpre, 0.1, 77, pre=pre)]
    ids = torch.randint(0, 10, (40960,), generator=g).to(dev)
    gt = r(40960, 512)
    out["embed token-table grad (V = 10)"] = lambda: [_table_grad(ids, gt, 10)]
    out["colsum groups (ragged 1090-row groups)"] = lambda: [colsum_groups(xd, 1090)]
    dyA, xA, dyB = r(16384, 1024), r(16384, 1024), r(16384, 4096)

    def grouped():
        outs = [torch.empty(1024, 1024, device=dev), torch.empty(4096, 1024, device=dev)]
        WG._launch([(dyB, xA, outs[1], 0.0), (dyA, xA, outs[0], 0.0)])
        return outs
    out["grouped tn (2 problems)"] = grouped
    return out


def bits(t):
    """bit patterns of a float tensor (NaN == NaN when the bits agree)"""
    if not t.is_floating_point():
        return t
    return t.view({4: torch.int32, 2: torch.int16}[t.element_size()])


def background(rank, ps, only, go, done):
    """BG=1, rank > 0: run this process's probes back to back (no checks) until
    rank 0 has finished, so one chosen kernel mix keeps running beside it"""
    import time
    if only and only.startswith("ubench:"):
        # one aggressor kernel class of tools/ubench/aggressor.hip instead of a probe
        import ctypes
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "aggressor.so"))
        mode = int(only.split(":")[1])
        buf = torch.zeros(4096, device="cuda")

        def agg():
            st = torch.cuda.current_stream().cuda_stream
            rc = lib.aggress(mode, 1024, 50000, ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(st))
            assert rc == 0, rc
        fns = [agg]
    else:
        fns = [fn for name, fn in ps.items() if not only or any(o in name for o in only.split(","))]
    n, t0 = 0, time.time()
    while not done.is_set() and time.time() - t0 < 300:
        for fn in fns:
            fn()
        n += 1
        if n == 2:
            go.set()
        torch.cuda.synchronize()
    go.set()
    print(f"[proc {rank}] background: {n} rounds of {len(fns)} probes", flush=True)


def worker(rank, q, go, done):
    torch.cuda.set_device(0)
    ps = probes("cuda")
    res = {}
    # ONLY<rank> / REPS<rank>: this process's own filter and count (e.g. proc 1
    # keeps one other kernel running beside proc 0's probe)
    only = os.environ.get(f"ONLY{rank}", os.environ.get("ONLY"))
    reps = int(os.environ.get(f"REPS{rank}", REPS))
    bg = os.environ.get("BG") == "1"
    if bg and rank > 0:
        background(rank, ps, only, go, done)
        q.put({})
        return
    if bg:
        go.wait(300)
    for name, fn in ps.items():
        if only and not any(o in name for o in only.split(",")):
            continue
        ref = [t.clone() if t is not None else None for t in fn()]
        bad = 0
        which = {}
        for _ in range(reps):
            got = fn()
            diff = False
            for i, (a, b) in enumerate(zip(got, ref)):
                if a is None or torch.equal(bits(a), bits(b)):
                    continue
                diff = True
                ne = bits(a) != bits(b)
                idx = ne.nonzero()
                w = which.setdefault(i, [0, 0, None, tuple(a.shape)])
                w[0] += 1
                w[1] = max(w[1], int(ne.sum()))
                if w[2] is None and len(idx):
                    w[2] = (idx[0].tolist(), idx[-1].tolist(), float((a.float() - b.float()).abs().max()),
                            int(torch.isnan(a[ne]).sum()), int(torch.isnan(b[ne]).sum()))
            bad += diff
        torch.cuda.synchronize()
        res[name] = bad
        print(f"[proc {rank}] {name}: {bad}/{reps} runs differ; per output (runs, max #elements, first/last index, "
              f"max |diff|, shape): {which}", flush=True)
    if rank == 0:
        done.set()
    q.put(res)


if __name__ == "__main__":
    n = int(os.environ.get("NPROC", "2"))
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    go, done = ctx.Event(), ctx.Event()
    ps = [ctx.Process(target=worker, args=(i, qq, go, done)) for i in range(n)]
    for p in ps:
        p.start()
    for _ in range(n):
        qq.get(timeout=600)
    for p in ps:
        p.join(60)
