#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2d
mkdir -p $O
timeout -k 10 240 python tools/bench_mgemm.py > $O/mgemm.txt 2>&1 || { cat $O/mgemm.txt; exit 1; }
V=base,gnodma
timeout -k 10 120 python tools/gemm_diag.py $V 16384 4096 1024 0 > $O/d1.txt 2>&1 || { cat $O/d1.txt; exit 1; }
cat $O/mgemm.txt $O/d1.txt | grep -v amdgpu.ids
