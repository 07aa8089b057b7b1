#!/bin/bash
# round 5: side-stream grouped weight gradients: engine tests, then C2 A/B SIDE=0 / SIDE=1
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r5h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wgrad.py tests/test_gpu_configs.py -k "wgrad or deferred or listener or c2" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  SIDE=0 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  SIDE=1 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
done
cat $O/ab.txt
