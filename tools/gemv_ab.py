"""Decode projection timing with COLD weights (csrc/gemv.hip): a hipGraph of
back-to-back packed GEMMs cycling over enough distinct weights (> 256 MB,
past the Infinity Cache) that every call streams its weights from HBM, as
in the decode step.  Per-call microseconds and weight GB/s per shape.
python tools/gemv_ab.py   (MTTS_LIB=... for tools/diag_build.sh variants)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mamba-tts-project_amd"))
import torch  # noqa: E402

from mtts import ops  # noqa: E402


def run(N, K, mode, reps=5):
    dev = "cuda"
    nw = max(8, int(384e6 // (N * K * 2)))
    ws = [ops.pack_rows_weight(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(nw)]
    x = torch.randn(32, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    kw = {}
    if mode in ("ln", "film"):
        kw["ln"] = (torch.ones(K, device=dev), torch.zeros(K, device=dev), 1e-5,
                    *((torch.randn(32, K, device=dev, dtype=torch.bfloat16),) * 2 if mode == "film" else (None, None)))
    if mode == "res":
        kw["res"] = torch.randn(32, N, device=dev, dtype=torch.bfloat16)

    def body():
        for w in ws:
            ops.gemm_rows(x, w, b, **kw)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * nw)
    print(f"N={N:5d} K={K:5d} {mode:5s} {us:6.2f} us/call  {N * K * 2 / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    for N, K, mode in [(4096, 1024, "ln"), (96, 2048, "plain"), (1024, 2048, "res"), (1024, 1024, "ln"),
                       (1024, 1024, "res"), (2048, 1024, "film"), (1024, 2048, "plain")]:
        run(N, K, mode)
