#!/bin/bash
# round 6: bitwise determinism of every training-step kernel of the probe under GPU sharing (2 processes, 20 reps)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6raceall
mkdir -p $O
cd $R
NPROC=2 REPS=${REPS:-20} timeout -k 10 900 python -u tools/dbg/race_probe.py > $O/race.txt 2>&1 || { tail -20 $O/race.txt; exit 1; }
grep "runs differ" $O/race.txt
