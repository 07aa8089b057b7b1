#!/bin/bash
# round-4 check 8: buffer-addressed c1 scan forward + attention K/V buffer
# loads: scan and attention parity, scan A/B vs the round-3 package, attention timing
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t8
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_attention.py -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  AB_ROOT=$R/tools/ab/base timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
  timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
SHAPES=C5m,C2 timeout -k 10 200 python tools/attn_ab.py > $O/attn.log 2>&1 || { tail $O/attn.log; exit 1; }
cat $O/attn.log
