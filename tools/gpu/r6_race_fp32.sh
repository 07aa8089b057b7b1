#!/bin/bash
# round 6: the fp32 scan-backward workspace probe alone, 1 process then 2
# processes sharing the GPU (is the rare carry difference tied to sharing?)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6racefp32
mkdir -p $O
cd $R
export ONLY="fp32 workspace" REPS=${REPS:-1500}
NPROC=1 timeout -k 10 400 python -u tools/dbg/race_probe.py > $O/n1.txt 2>&1 || { tail -20 $O/n1.txt; exit 1; }
grep "runs differ" $O/n1.txt
NPROC=2 timeout -k 10 400 python -u tools/dbg/race_probe.py > $O/n2.txt 2>&1 || { tail -20 $O/n2.txt; exit 1; }
grep "runs differ" $O/n2.txt
