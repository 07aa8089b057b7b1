#!/bin/bash
# round-4 check 23: attention forward / backward at 4096 / 5120 / 6144 queries
# (C5m keys): is the workgroup-round tail visible?
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t23
mkdir -p $O
cd $R
for i in 1 2; do
  SHAPES=C5m4k,C5m,C5m6k timeout -k 10 200 python tools/attn_ab.py >> $O/attn.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/attn.txt
