#!/bin/bash
# mtts_gemm correctness + speed vs hipBLASLt on the C2 shapes
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2c
mkdir -p $O
timeout -k 10 240 python tools/bench_mgemm.py > $O/mgemm.txt 2>&1; rc=$?
cat $O/mgemm.txt | grep -v amdgpu.ids
exit $rc
