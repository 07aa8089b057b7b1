#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2l
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
MTTS_C1_SPREAD=1 timeout -k 10 300 $PT tests/test_gpu_ops.py -m gpu -k "c1" > $O/c1_tests.log 2>&1; rc=$?
tail -3 $O/c1_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/scan_ab.py xl spread > $O/ab.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/ab.txt
exit $rc
