#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2d
mkdir -p $O
V=base,gfixk,gnodma
timeout -k 10 120 python tools/gemm_diag.py $V 16384 4096 1024 0 > $O/d1.txt 2>&1 || { cat $O/d1.txt; exit 1; }
timeout -k 10 120 python tools/gemm_diag.py $V 16384 1024 4096 0 > $O/d2.txt 2>&1 || { cat $O/d2.txt; exit 1; }
cat $O/d1.txt $O/d2.txt | grep -v amdgpu.ids
