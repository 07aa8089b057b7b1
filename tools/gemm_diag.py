"""Interleaved timing of mtts_gemm across timing-only builds (tools/diag_build.sh
NAME "-D..." gemm.hip) in ONE process: each libmtts_<name>.so is loaded with
ctypes and called on the same operands.
  python tools/gemm_diag.py base,gnodma,... [m n k] [layout]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import _lib as L  # noqa: E402

names = sys.argv[1].split(",")
m, n, k = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (16384, 4096, 1024)
layout = int(sys.argv[5]) if len(sys.argv) > 5 else 0
libs = {}
for nm in names:
    base = nm.split("@")[0]     # name@G: run with MTTS_GEMM_GROUP=G
    path = os.path.join(ROOT, "mamba-tts-project_amd", "mtts", "libmtts.so" if base == "base" else f"libmtts_{base}.so")
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    lib.mtts_gemm.argtypes = [C.POINTER(L.GemmArgs), C.c_void_p]
    lib.mtts_gemm.restype = C.c_int
    libs[nm] = lib

rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
args = L.GemmArgs()
if layout == 0:
    a, b = rnd(m, k), rnd(n, k)
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    args.lda, args.ldb, args.ldc, args.out_dtype = k, k, n, 1
else:
    a, b = rnd(k, m), rnd(k, n)
    c = torch.empty(m, n, device="cuda", dtype=torch.float32)
    args.lda, args.ldb, args.ldc, args.out_dtype = m, n, n, 0
args.m, args.n, args.k, args.layout, args.splits = m, n, k, layout, 1
args.a, args.b, args.c = a.data_ptr(), b.data_ptr(), c.data_ptr()
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
fl = 2 * m * n * k
res = {nm: [] for nm in names}
for rnd_i in range(5):
    for nm, lib in libs.items():
        if "@" in nm:
            os.environ["MTTS_GEMM_GROUP"] = nm.split("@")[1]
        else:
            os.environ.pop("MTTS_GEMM_GROUP", None)
        for _ in range(3):
            lib.mtts_gemm(C.byref(args), stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            assert lib.mtts_gemm(C.byref(args), stream) == 0
        e1.record()
        e1.synchronize()
        res[nm].append(e0.elapsed_time(e1) / 20)
for nm, v in res.items():
    v.sort()
    print(f"{nm:10s} median {v[2] * 1e3:8.1f} us  min {v[0] * 1e3:8.1f} us  {fl / v[2] / 1e9:6.0f} TF/s", flush=True)
