#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2i
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_ops.py -m gpu -k "rows" > $O/rows_tests.log 2>&1; rc=$?
tail -15 $O/rows_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 $PT tests/test_gpu_modules.py -m gpu > $O/mod_tests.log 2>&1; rc=$?
tail -3 $O/mod_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/decode_ab.py shapes splitk prefetch > $O/decode_ab.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/decode_ab.txt
exit $rc
