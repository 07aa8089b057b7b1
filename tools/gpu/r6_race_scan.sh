#!/bin/bash
# round 6: the scan-backward probes only, more repetitions (2 processes x 60)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6racescan
mkdir -p $O
cd $R
NPROC=2 REPS=60 ONLY="scan bwd" timeout -k 10 900 python -u tools/dbg/race_probe.py > $O/race.txt 2>&1 || { tail -20 $O/race.txt; exit 1; }
grep "runs differ" $O/race.txt
