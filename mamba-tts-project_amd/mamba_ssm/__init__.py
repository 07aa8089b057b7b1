"""`mamba_ssm` import surface backed by libmtts (MI355X).

The reference imports `from mamba_ssm import Mamba` (mamba_decoder.py:4) and
relies on the documented contract `out, state = mamba(x[, state])`
(mamba_decoder.py:10-15).  With mamba-tts-project_amd/ on sys.path, that
import resolves here, so even the reference's own mamba_decoder.py runs on the
HIP kernels.  Upstream op names are provided for code that calls them
directly (mamba_ssm.ops.selective_scan_interface / causal_conv1d style).
"""
from mtts.mamba import Mamba  # noqa: F401
from mtts.ops import (  # noqa: F401
    causal_conv1d_fn,
    causal_conv1d_update,
    selective_scan_fn,
    selective_state_update,
)

__all__ = ["Mamba", "selective_scan_fn", "selective_state_update", "causal_conv1d_fn", "causal_conv1d_update"]
