"""A/B timing of selective_scan_fwd variants at the north-star and C2 shapes.
python tools/scan_ab.py   (env MTTS_LIB selects a library build)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch
import bench
variants = [("v2", {}), ("v1", {"MTTS_SCAN_FWD_V1": "1"})]
if len(sys.argv) > 1:
    variants = [v for v in variants if v[0] in sys.argv[1:]]
for dtype in (torch.bfloat16, torch.float32):
    for name, env in variants:
        for k in ("MTTS_SCAN_FWD_V1",):
            os.environ.pop(k, None)
        os.environ.update(env)
        ms, nb, bw = bench.scan_roofline(dtype, iters=10)
        print(f"{name} {str(dtype)[6:]} north-star {ms:.3f} ms {bw/1e9:.0f} GB/s ({bw/8e12*100:.1f}% of 8 TB/s)", flush=True)
        ms, nb, bw = bench.scan_roofline(dtype, B=8, L=2048, D=2048, iters=20)
        print(f"{name} {str(dtype)[6:]} C2 shape   {ms:.3f} ms {bw/1e9:.0f} GB/s", flush=True)
