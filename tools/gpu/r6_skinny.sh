#!/bin/bash
# round 6: x_proj forward SKINNY_N vs hipBLASLt -- per-op timings and C2 steps with / without it
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6sk
mkdir -p $O
cd $R
timeout -k 10 600 python -u tools/skinny_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
