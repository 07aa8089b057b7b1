#!/bin/bash
# rocprofv3 kernel stats of the default bench command and of 60 decode steps
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $O
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o b -- python3 $GRAFT_REPO_ROOT/bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
tail -1 $O/bench.log | cut -c1-300
DEC_STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_ab.py rowsonly > $O/dec.log 2>&1 || { tail -5 $O/dec.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
