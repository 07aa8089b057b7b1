"""Run the C5-shape decoder bench once (for rocprofv3)."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import bench  # noqa: E402
print(json.dumps(bench.c5_step_bench(0, 1, "cuda", steps=2)))
