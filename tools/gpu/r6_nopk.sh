#!/bin/bash
# round 6: scan backward kernels without packed-f32 ops -- scan parity tests,
# the background-MFMA race probe, then same-box timing against tools/ab/base
# (the committed library: packed ops): scan kernels and the C2 step
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUTD:-r6nopk}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "scan" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
OUT=${OUTD:-r6nopk}/race MIXES="ubench:1;skinny tn;attn" ONLY0="workspace,one segment,scan bwd C2 (du" REPS0=200 \
  timeout -k 10 600 bash tools/gpu/r6_race_bg.sh > $O/race.txt 2>&1 || { tail -5 $O/race.txt; exit 1; }
grep -E "==|differ" $O/race.txt | cut -c1-160
for i in 1 2 3; do
  echo "== base" >> $O/ab.txt; AB_ROOT=tools/ab/base timeout -k 10 300 python tools/scan_lib_ab.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== new" >> $O/ab.txt; timeout -k 10 300 python tools/scan_lib_ab.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
done
for i in 1 2 3; do
  echo "== base" >> $O/c2.txt; AB_ROOT=tools/ab/base SIDE=0 timeout -k 10 300 python tools/c2_ab.py >> $O/c2.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== new" >> $O/c2.txt; SIDE=0 timeout -k 10 300 python tools/c2_ab.py >> $O/c2.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/ab.txt $O/c2.txt
