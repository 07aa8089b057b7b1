#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2g
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_gemm.py -m gpu > $O/gemm_tests.log 2>&1; rc=$?
tail -3 $O/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python tools/bench_mgemm.py ff1,ff2 > $O/mgemm.txt 2>&1 || { cat $O/mgemm.txt; exit 1; }
grep -v amdgpu.ids $O/mgemm.txt
timeout -k 10 300 python tools/gemm_step_ab.py > $O/step.txt 2>&1; rc=$?
tail -1 $O/step.txt
exit $rc
