#!/bin/bash
# round 6: bitwise determinism of the round-6 kernels under GPU sharing (2 processes, 30 reps each)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6race
mkdir -p $O
cd $R
NPROC=2 REPS=30 ONLY="dropout,embed,colsum groups,grouped" timeout -k 10 600 python -u tools/dbg/race_probe.py > $O/race.txt 2>&1 || { tail -20 $O/race.txt; exit 1; }
grep "runs differ" $O/race.txt
