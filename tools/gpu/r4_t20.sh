#!/bin/bash
# round-4 check 20: segment sweep of the scan backward for this tree and the base
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t20
mkdir -p $O
cd $R
for i in 1 2; do
  AB_ROOT=tools/ab/base SWEEP="scan_bwd_segs=4,6" timeout -k 10 200 python tools/scan_lib_ab.py >> $O/sweep.jsonl 2>>$O/err || { tail $O/err; exit 1; }
  SWEEP="scan_bwd_segs=4,6" timeout -k 10 200 python tools/scan_lib_ab.py >> $O/sweep.jsonl 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/sweep.jsonl
