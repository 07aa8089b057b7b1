#!/bin/bash
# C2 step: in-process routing A/B and a kernel-trace of the default routing
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2r
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_step_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
