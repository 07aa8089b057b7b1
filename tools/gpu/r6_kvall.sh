#!/bin/bash
# round 6: K/V batching parity (incl. a retained-graph double backward) and the decoder / DP tests around it
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6kva
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread \
  tests/test_gpu_kvall.py tests/test_gpu_wgrad.py tests/test_gpu_c5.py tests/test_gpu_c5_dp.py tests/test_gpu_modules.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
