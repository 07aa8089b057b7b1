#!/bin/bash
# round-4 check 25: attention softmax max as raw v_max3 tree (no quieting passes)
# attention + C5 parity, forward A/B against tools/ab/base
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t25
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_c5.py -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  echo base >> $O/attn.txt; AB_ROOT=tools/ab/base SHAPES=C2,C5m timeout -k 10 120 python tools/attn_ab.py >> $O/attn.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo new >> $O/attn.txt; SHAPES=C2,C5m timeout -k 10 120 python tools/attn_ab.py >> $O/attn.txt 2>>$O/err || { tail $O/err; exit 1; }
done
grep -E "^(base|new)|fwd [0-9]" $O/attn.txt
