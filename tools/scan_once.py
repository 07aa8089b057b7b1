"""Run selective_scan_fwd at the north-star shape a few times (for rocprofv3).
python tools/scan_once.py [fp32|bf16]; SCAN_PATH=<n> forces a forward kernel
(mtts_set_override MTTS_OVR_SCAN_PATH: 1 c1, 2 w2)."""
import contextlib
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from mtts import _lib  # noqa: E402
dtype = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == "fp32") else torch.bfloat16
path = os.environ.get("SCAN_PATH")
with (_lib.override(scan_path=int(path)) if path else contextlib.nullcontext()):
    ms, nbytes, bw = bench.scan_roofline(dtype, iters=int(os.environ.get("ITERS", "5")))
print(f"scan {dtype} path {path} {ms:.3f} ms  {nbytes} B  {bw/1e9:.0f} GB/s")
