#!/bin/bash
# C2-shape scan forward (B=8, L=2048, D=2048): automatic plan vs forced L-segment counts
set -e -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep "fwd.*bfloat16" | sed "s/^/segs=auto /"
  for k in 1 2 4; do
    MTTS_SCAN_SEGS=$k timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep "fwd.*bfloat16" | sed "s/^/segs=$k /"
  done
done
