#!/bin/bash
# C2 step: GEMM routing A/B (hip / wgrad-only / hipBLASLt, interleaved) and bench eager vs hipGraph
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_step_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
for g in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --skip-extras --graph $g > $O/bench_g$g.json 2> $O/bench_g$g.err
  echo "graph=$g $(grep -o '"ms_per_step": [0-9.]*' $O/bench_g$g.json)"
done
