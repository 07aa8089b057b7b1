"""bench.py's N-rank launch on CPU: `python bench.py --gpus 2` without a
launcher starts torch.distributed.run with 2 ranks as a child process, the
ranks join one process group (gloo here; RCCL on the GPU node), time a
barrier-bracketed region, take the max over ranks and rank 0 prints one JSON
line with n_gpus = 2 (--launch-check: the plumbing without GPU work)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = dict(os.environ, MTTS_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_launches_two_ranks():
    rec = _run(2)
    assert rec["n_gpus"] == 2 and rec["allreduce_ok"] and rec["steps"] == 3 and rec["warmup"] == 1
    # the N > 1 line explains itself: backward time, the all-reduce time left
    # exposed after it, and the bucket layout (bench.py dp_breakdown)
    dp = rec["dp"]
    assert dp["backward_ms"] >= 0 and dp["allreduce_exposed_ms"] >= 0 and dp["steps"] == 3
    assert dp["buckets"] >= 2 and len(dp["bucket_MB"]) == dp["buckets"] and dp["grad_MB"] > 0
    assert dp["comm_dtype"] == "float32" and dp["reduce_op"] in ("avg", "sum+scale")


def test_bench_single_rank_needs_no_launcher():
    assert _run(1)["n_gpus"] == 1
