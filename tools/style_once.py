"""Run the style-pipeline bench leg once (for rocprofv3): bench.style_bench."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import bench  # noqa: E402
print(json.dumps(bench.style_bench(iters=5)))
