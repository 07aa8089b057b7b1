"""mtts — MI355X (gfx950) kernels + host modules for the MambaTTSDecoder hot path.

Layout:
  csrc/            HIP kernels and the C ABI (include/mtts.h) -> libmtts.so
  _lib.py          ctypes binding (no CPU fallback: missing library = error)
  ops.py           tensor wrappers + autograd Functions (scan, conv1d, step, LN/FiLM)
  mamba.py         Mamba mixer (replacement for mamba_ssm.Mamba, documented contract)
  attention.py     nn.MultiheadAttention-compatible cross-attention
  attn_kernels.py  attention core
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
