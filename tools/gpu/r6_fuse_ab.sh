#!/bin/bash
# round 6: same-box C2 step A/B -- base (tools/ab/base: K/V rows submitted by KVAllFn), this tree with the
# bias column sums separate (FUSE=0) and summed inside the TN kernel (FUSE=1); three interleaved rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fab
mkdir -p $O
cd $R
for i in 1 2 3; do
  echo "== base" >> $O/ab.txt; AB_ROOT=tools/ab/base SIDE=0 timeout -k 10 300 python tools/c2_ab.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== fuse0" >> $O/ab.txt; FUSE=0 SIDE=0 timeout -k 10 300 python tools/c2_ab.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== fuse1" >> $O/ab.txt; FUSE=1 SIDE=0 timeout -k 10 300 python tools/c2_ab.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/ab.txt
