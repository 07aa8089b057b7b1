#!/bin/bash
# parity tests of the paths a change touches, then the C2 step: eager and hipGraph, twice each
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3step
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for g in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --skip-extras --graph $g > $O/bench_g$g.json 2> $O/bench_g$g.err || { tail -20 $O/bench_g$g.err; exit 1; }
  echo "graph=$g $(grep -o '"ms_per_step": [0-9.]*' $O/bench_g$g.json)"
done
