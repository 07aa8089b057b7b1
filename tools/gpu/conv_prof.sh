#!/bin/bash
# kernel-level times of the conv kernels (tiled vs untiled) at the C2 shape
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/convprof
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
cat $O/kt/kt_kernel_stats.csv | cut -d, -f1-8 | head -20
