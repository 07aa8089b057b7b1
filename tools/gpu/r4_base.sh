#!/bin/bash
# Round-4 baseline on a fresh box: default bench line + kernel trace of 5 C2 steps.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4base
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o kt -- python3 $R/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O -name "*kernel_trace.csv" -size +20M -delete; find $O -name "*.db" -delete; du -sh $O
