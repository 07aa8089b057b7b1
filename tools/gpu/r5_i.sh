#!/bin/bash
# round 5: skinny weight gradients in the grouped launch: tests, then C2 A/B vs base
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r5i}
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wgrad.py tests/test_gpu_configs.py tests/test_gpu_modules.py tests/test_gpu_c5.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  AB_ROOT=tools/ab/base timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
done
cat $O/ab.txt
