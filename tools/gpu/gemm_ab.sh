#!/bin/bash
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/gemm_pp_ab.py 2>&1 | tee $O/ab.log
