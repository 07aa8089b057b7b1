#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2n
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $PT tests -m gpu > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_step_ab.py > $O/step.txt 2>&1; rc=$?
tail -1 $O/step.txt
exit $rc
