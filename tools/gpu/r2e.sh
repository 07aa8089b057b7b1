#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2e
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_gemm.py -m gpu > $O/gemm_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/gemm_tests.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_step_ab.py > $O/step.txt 2>&1; rc=$?
tail -5 $O/step.txt
exit $rc
