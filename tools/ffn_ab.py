"""C2 training step A/B of the FFN path, interleaved in one process:
fused bias+GELU / GELU-backward epilogues on the one-tile-per-workgroup
ping-pong kernel (MTTS_GEMM_PP=1, default), the same on the persistent
ping-pong kernel (PP=2: a tile's epilogue overlaps the next tile's main loop),
and the unfused FFN (NT GEMMs + torch GELU kernels)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from mtts import gemm as G  # noqa: E402

import skinny_ab as S  # noqa: E402  (builds the C2 model and its step())

res = {"fused pp1": [], "fused pp2": [], "unfused": []}
for _ in range(3):
    for kind in res:
        G.FFN_FUSED = kind != "unfused"
        os.environ["MTTS_GEMM_PP"] = "2" if kind == "fused pp2" else "1"
        res[kind].append(S.timeit())
os.environ.pop("MTTS_GEMM_PP")
G.FFN_FUSED = True
print({k: [round(x, 2) for x in v] for k, v in res.items()}, flush=True)
