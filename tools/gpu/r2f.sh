#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2f
mkdir -p $O
cd /tmp
for m in hip blaslt; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- python $GRAFT_REPO_ROOT/tools/gemm_step_ab.py $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
done
find $O -name "*stats*"
