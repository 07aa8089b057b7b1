"""Run selective_scan_fwd at the north-star shape a few times (for rocprofv3)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch
import bench
dtype = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == "fp32") else torch.bfloat16
ms, nbytes, bw = bench.scan_roofline(dtype, iters=int(os.environ.get("ITERS", "5")))
print(f"scan {dtype} {ms:.3f} ms  {nbytes} B  {bw/1e9:.0f} GB/s")
