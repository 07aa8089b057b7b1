#!/bin/bash
# round-4 check 26: attention dK/dV kernel with two slices of Q / dO loads in
# flight: parity (this tree: 3 waves per SIMD, 5 spills), then backward A/B of
# base / this tree / tools/ab/v2 (same code at 2 waves per SIMD, no spills)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t26
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_c5.py -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for t in tools/ab/base . tools/ab/v2; do
    echo "== $t" >> $O/attn.txt; AB_ROOT=$t SHAPES=C5m timeout -k 10 120 python tools/attn_ab.py >> $O/attn.txt 2>>$O/err || { tail $O/err; exit 1; }
  done
done
grep -E "^==|bwd" $O/attn.txt
