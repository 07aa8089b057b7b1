"""Hand-written bf16 MFMA GEMMs (csrc/gemm.hip, `mtts_gemm`) for the
decoder's training projections (reference mamba_decoder.py:29-43, applied at
:61-88): forward x·Wᵀ and data gradient dy·W in the NT layout (both operands
k-contiguous; the data gradient reads the cast kernel's Wᵀ copy), weight
gradient dyᵀ·x in the TN layout straight into the fp32 master gradient.

Epilogues run on the fp32 accumulator: bias, GELU (writing the bf16
pre-activation for the backward) and the GELU backward fused into the data
gradient of the FFN's second projection.
"""
from __future__ import annotations

import torch

from . import _lib as L

EPI_BIAS, EPI_GELU, EPI_DGELU = 1, 2, 4
NT, TN = 0, 1
TILE = 256
ENABLED = True   # routing switch for in-process A/B timing (tools/gemm_step_ab.py)
FFN_FUSED = True   # FFN with bias + GELU fused into the first GEMM's epilogue and the GELU
#                    backward into the second's data gradient (linear.ffn)


def _rowmajor(t):
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


def nt_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Shapes/layouts the NT kernel takes: bf16, k % 64 == 0, n % 8 == 0."""
    return (ENABLED and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.is_cuda
            and _rowmajor(a) and _rowmajor(b)
            and a.shape[1] == b.shape[1] and a.shape[1] % 64 == 0 and b.shape[0] % 8 == 0 and a.shape[0] > 0)


def epi_ok(bias: torch.Tensor = None, aux: torch.Tensor = None) -> bool:
    """Epilogue operand alignment the kernel reads with (mirrors mtts_gemm's
    checks): fp32 bias 16-byte, bf16 bias 8-byte aligned; the GELU /
    GELU-backward aux rows 8-byte aligned with ld_aux % 4 == 0."""
    if bias is not None and bias.data_ptr() % (16 if bias.dtype == torch.float32 else 8) != 0:
        return False
    if aux is not None and (aux.data_ptr() % 8 != 0 or aux.stride(0) % 4 != 0 or aux.stride(-1) != 1):
        return False
    return True


def tn_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (ENABLED and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.is_cuda
            and _rowmajor(a) and _rowmajor(b)
            and a.shape[0] == b.shape[0] and a.shape[0] % 64 == 0 and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0)


def mm_nt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor = None, gelu_aux: torch.Tensor = None,
          dgelu_aux: torch.Tensor = None, out: torch.Tensor = None) -> torch.Tensor:
    """bf16 C[m,n] = a[m,k] · b[n,k]ᵀ (+bias) with an optional GELU epilogue
    (gelu_aux receives the pre-activation, C = gelu of it) or GELU-backward
    epilogue (C = bf16(AB) · gelu'(dgelu_aux))."""
    m, k = a.shape
    n = b.shape[0]
    if not epi_ok(bias, gelu_aux if gelu_aux is not None else dgelu_aux):
        raise ValueError("mm_nt: bias / aux not aligned for the epilogue's vector accesses (gemm.epi_ok)")
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=torch.bfloat16)
    args = L.GemmArgs()
    args.m, args.n, args.k, args.layout, args.splits, args.out_dtype = m, n, k, NT, 1, 1
    epi = 0
    if bias is not None:
        epi |= EPI_BIAS
        args.bias, args.bias_dtype = bias.data_ptr(), L.dtype_code(bias)
    aux = gelu_aux if gelu_aux is not None else dgelu_aux
    if gelu_aux is not None:
        epi |= EPI_GELU
    if dgelu_aux is not None:
        epi |= EPI_DGELU
    if aux is not None:
        args.aux, args.ld_aux = aux.data_ptr(), aux.stride(0)
    args.epilogue = epi
    args.lda, args.ldb, args.ldc = a.stride(0), b.stride(0), out.stride(0)
    args.a, args.b, args.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
    L.call("mtts_gemm", args)
    return out


def tn_splits(m: int, n: int, k: int) -> int:
    """Split-K factor for the weight gradient: fill >= ~256 workgroups while
    each split keeps >= 1024 of the reduction (C2: in_proj 4, out_proj / FFN
    8, q / o projections 16; tools/bench_mgemm.py); with fewer than 64 output
    tiles a split may go down to 256 (C2's text K/V projection, 1024 tokens x
    32 tiles: 4 splits instead of 32 workgroups on 256 CUs)."""
    tiles = -(-m // TILE) * -(-n // TILE)
    min_k = 1024 if tiles >= 64 else 256
    s = 1
    while tiles * s < 256 and k % (64 * s * 2) == 0 and k // (s * 2) >= min_k:
        s *= 2
    return s


def mm_tn(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, beta: float = 0.0,
          splits: int = None) -> torch.Tensor:
    """fp32 C[m,n] = a[k,m]ᵀ · b[k,n] (+ beta·C): the weight gradient dyᵀ·x."""
    k, m = a.shape
    n = b.shape[1]
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=torch.float32)
    args = L.GemmArgs()
    s = tn_splits(m, n, k) if splits is None else splits
    args.m, args.n, args.k, args.layout, args.splits, args.out_dtype = m, n, k, TN, s, 0
    args.lda, args.ldb, args.ldc = a.stride(0), b.stride(0), out.stride(0)
    args.a, args.b, args.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
    args.beta = beta
    ws = None
    if s > 1:
        ws = torch.empty(L.lib().mtts_gemm_workspace(args), device=a.device, dtype=torch.uint8)
        args.workspace = ws.data_ptr()
    L.call("mtts_gemm", args)
    return out


# ------------------------------------------------------------------ skinny GEMMs (csrc/skinny.hip)
SKINNY_N, SKINNY_SMALL_K = 0, 1
SKINNY = True   # routing switch (in-process A/B: tools/skinny_ab.py)
SKINNY_TN_KERNEL = True  # x_proj / dt_proj weight gradients on the SKINNY_TN kernel (mamba.py; skinny_tn_ok)
WGRAD_SKINNY_ON_TN = False  # linear.wgrad: skinny weight gradients on the big TN kernel (35.5 vs 33.7 us: off)
# x_proj forward on SKINNY_N: round 3 measured 25 vs 21 us for hipBLASLt, round 5
# 24.5-25.8 vs 24.2 us (profiles/r05_skinny_n_*_ab.txt), round 6 25.6 vs 19.9 us
# per call and C2 steps 33.63 / 33.71 / 33.55 vs 33.47 / 33.61 / 33.53 ms
# (profiles/r06_skinny_xproj_ab.txt): hipBLASLt stays the x_proj forward
SKINNY_XPROJ = False
# dt_proj forward and the x_proj data gradient (du += d(x_dbl) W_x) on the
# skinny kernels (SMALL_K); per call 22.9 / 37.3 us vs 21.5 / 31.7 for
# hipBLASLt in round 6 (tools/skinny_ab.py ops), but C2 steps equal either
# way (32.68-32.72 vs 32.69-32.75 ms, profiles/r06_skinny_xproj_ab.txt): kept
SKINNY_DTPROJ = True
SKINNY_DU = True


def _skinny_operand(t):
    return (t.dim() == 2 and t.dtype == torch.bfloat16 and t.is_cuda and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0)


def skinny_ok(a: torch.Tensor, b: torch.Tensor, out_dtype=torch.bfloat16, out: torch.Tensor = None) -> bool:
    """a (m, k) . b (n, k)^T on csrc/skinny.hip: bf16 k-contiguous operands,
    k % 32 == 0, n % 4 == 0, and either n <= 128 or k <= 128 (SMALL_K with a
    bf16 C: n % 8 == 0 and 16-byte C rows)."""
    if not (SKINNY and _skinny_operand(a) and _skinny_operand(b) and a.shape[1] == b.shape[1]):
        return False
    m, k = a.shape
    n = b.shape[0]
    if m == 0 or k % 32 or n % 4 or not (n <= 128 or k <= 128):
        return False
    if out is not None:
        out_dtype = out.dtype
        es = 4 if out.dtype == torch.float32 else 2
        if (out.dtype not in (torch.float32, torch.bfloat16) or out.stride(1) != 1 or out.stride(0) % 4
                or out.data_ptr() % (4 * es) or tuple(out.shape) != (m, n)):
            return False
    if n > 128 and out_dtype == torch.bfloat16:
        # SMALL_K's bf16 stores move 8 columns (16 bytes) per lane (mtts_gemm_skinny)
        if n % 8 or (out is not None and (out.stride(0) % 8 or out.data_ptr() % 16)):
            return False
    return out_dtype in (torch.float32, torch.bfloat16)


def mm_skinny(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, beta: float = 0.0,
              out_dtype=torch.bfloat16) -> torch.Tensor:
    """C[m, n] = a[m, k] . b[n, k]^T (+ beta C) with fp32 accumulation; the
    SKINNY_N kernel for n <= 128, else SMALL_K (k <= 128)."""
    m, k = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=out_dtype)
    args = L.SkinnyArgs()
    args.mode = SKINNY_N if n <= 128 else SKINNY_SMALL_K
    args.m, args.n, args.k = m, n, k
    args.c_dtype = L.dtype_code(out)
    args.beta = beta
    args.lda, args.ldb, args.ldc = a.stride(0), b.stride(0), out.stride(0)
    args.a, args.b, args.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
    L.call("mtts_gemm_skinny", args)
    return out


SKINNY_TN_MODE = 2


def skinny_tn_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """a (k, m) wide (m % 128 == 0), b (k, n) narrow (n <= 128, n % 8 == 0),
    both token-major bf16 with 16-byte rows: the SKINNY_TN weight gradient."""
    return (SKINNY and SKINNY_TN_KERNEL and _skinny_operand(a) and _skinny_operand(b) and a.shape[0] == b.shape[0] and a.shape[0] > 0
            and a.shape[1] % 128 == 0 and b.shape[1] <= 128 and b.shape[1] % 8 == 0)


def mm_skinny_tn(a: torch.Tensor, b: torch.Tensor, trans_c: bool = False) -> torch.Tensor:
    """fp32 a^T b (m x n), or its transpose (n x m) with trans_c, on the
    SKINNY_TN kernel (chunk partials summed in fixed order)."""
    k, m = a.shape
    n = b.shape[1]
    out = torch.empty((n, m) if trans_c else (m, n), device=a.device, dtype=torch.float32)
    args = L.SkinnyArgs()
    args.mode, args.m, args.n, args.k = SKINNY_TN_MODE, m, n, k
    args.c_dtype, args.beta, args.trans_c = L.F32, 0.0, int(trans_c)
    args.lda, args.ldb, args.ldc = a.stride(0), b.stride(0), out.stride(0)
    args.a, args.b, args.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
    ws = torch.empty(L.lib().mtts_gemm_skinny_workspace(args), device=a.device, dtype=torch.uint8)
    args.workspace = ws.data_ptr()
    L.call("mtts_gemm_skinny", args)
    return out
