#!/bin/bash
# round-4 check 28: LayerNorm backward rows per workgroup (override ln_rb):
# LN parity under each value, then timing
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t28
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "layernorm or ln" -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 120 python tools/bench_ln.py >> $O/ln.txt 2>>$O/err || { tail $O/err; exit 1; }; done
cat $O/ln.txt
