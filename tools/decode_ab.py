"""Decode-step A/B: HIP skinny GEMM (csrc/rows.hip) vs hipBLASLt for the
C4 projections, per shape and for the whole graph-replayed decode step.
python tools/decode_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mamba-tts-project_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from mtts import ops  # noqa: E402
from mtts.decode import DecodeEngine  # noqa: E402


def t_us(fn, iters=50, reps=20):
    """per-call time from a hipGraph of `iters` back-to-back calls (launch overhead excluded)"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * reps)


def shapes():
    dev = "cuda"
    for (N, K) in [(4096, 1024), (96, 2048), (2048, 64), (1024, 2048), (1024, 1024), (2048, 1024), (10, 1024)]:
        x = torch.randn(32, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        wp = ops.pack_rows_weight(w)
        tp = t_us(lambda: ops.gemm_rows(x, wp, b))
        t1 = t_us(lambda: ops.gemm_rows(x, w, b))
        tb = t_us(lambda: torch.addmm(b, x, w.t()))
        gbs = N * K * 2 / tp / 1e3
        print(f"N={N:5d} K={K:5d}  packed {tp:6.2f} us ({gbs:6.0f} GB/s)  rows {t1:6.2f} us   "
              f"hipBLASLt {tb:6.2f} us", flush=True)


def step(modes=(True, False)):
    import mamba_decoder
    c = dict(bench.C2)
    dev = "cuda"
    torch.manual_seed(0)
    m = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"],
                                      n_heads=c["n_heads"], d_ff=c["d_ff"], d_style=c["d_style"]).to(dev).eval()
    m.compute_dtype = torch.bfloat16
    c["B"] = 32
    _, text, z, mask = bench.make_batch(c, dev, 7)
    res = {}
    n = int(os.environ.get("DEC_STEPS", 300))
    for rows in (modes if n < 300 else modes + modes):
        m._engine = DecodeEngine(m, use_graph=True, use_rows=rows)
        tok = torch.zeros(32, 1, dtype=torch.long, device=dev)
        states = [None] * c["n_layers"]
        lat = []
        with torch.no_grad():
            for t in range(n):
                t0 = time.perf_counter()
                lg, states = m.decode_step(tok, text, z, states, t, text_mask=mask)
                tok = lg.argmax(-1)
                torch.cuda.synchronize()
                lat.append((time.perf_counter() - t0) * 1e3)
        lat = sorted(lat[n // 3:])
        res.setdefault(rows, []).append(lat[len(lat) // 2])
    print({("rows" if k else "hipBLASLt"): v for k, v in res.items()}, "p50 ms", flush=True)


DEFAULTS = dict(DecodeEngine.OPTIONS)

if __name__ == "__main__":
    what = sys.argv[1:] or ["shapes", "step"]
    if "shapes" in what:
        shapes()
    if "step" in what:
        step()
    if "rowsonly" in what:
        step((True,))
    # DecodeEngine.OPTIONS A/B, interleaved: python tools/decode_ab.py opt:packed
    for w in what:
        if w.startswith("opt:"):
            key = w[4:]
            for _ in range(2):
                for v in (True, False):
                    DecodeEngine.OPTIONS[key] = v
                    print(key, v, end=" ", flush=True)
                    step((True,))
            DecodeEngine.OPTIONS[key] = DEFAULTS[key]
    if "splitk" in what:   # rows kernels with / without the cross-workgroup K split, interleaved
        for _ in range(2):
            for sk in (True, False):
                ops.ROWS_SPLITK = sk
                print("splitk", sk, end=" ", flush=True)
                step((True,))
        ops.ROWS_SPLITK = True
