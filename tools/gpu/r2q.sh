#!/bin/bash
# GEMM bf16 epilogue: parity + in-process A/B of dwordx4 vs dwordx2 stores
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2q
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_epi_ab.py 5 2>&1 | tee $O/ab.log
