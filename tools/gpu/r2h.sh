#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2h
mkdir -p $O
timeout -k 10 300 python tools/gemm_step_ab.py > $O/step.txt 2>&1; rc=$?
tail -1 $O/step.txt
exit $rc
