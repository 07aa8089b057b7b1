#!/bin/bash
# round-4 check 31: w2 forward: exp products first, y chains interleaved; reduce-scatter DPP sources formed first
# scan + decoder parity, scan A/B against tools/ab/base
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t31
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_configs.py -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  AB_ROOT=tools/ab/base timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
  timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
