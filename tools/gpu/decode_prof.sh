#!/bin/bash
# kernel stats of the C4 decode step (graph replay, tools/decode_ab.py rowsonly)
set -e -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/decprof
mkdir -p $O
cd /tmp
DEC_STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o dec -- python3 $R/tools/decode_ab.py rowsonly > $O/dec.log 2>&1 || { tail -20 $O/dec.log; exit 1; }
find $O -name "*.db" -delete
ls $O
