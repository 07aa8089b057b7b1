#!/bin/bash
# round-4 check 18: C2 scan forward / backward segment-count and path sweeps
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t18
mkdir -p $O
cd $R
for i in 1 2; do
  SWEEP="scan_bwd_segs=1,2,3,4,6,8;scan_segs=1,2,3,4;scan_path=1,2" timeout -k 10 200 python tools/scan_lib_ab.py >> $O/sweep.jsonl 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/sweep.jsonl
