#!/bin/bash
# round 6: dQ LDS-DMA form -- parity, then same-process A/B and a kernel trace of both
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6dq
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -q -m gpu -x --timeout 200 --timeout-method thread tests/test_gpu_attention.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python tools/attn_dq_ab.py > $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
cat $O/ab.txt
