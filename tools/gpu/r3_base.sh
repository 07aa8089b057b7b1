#!/bin/bash
# full -m gpu suite, default bench line, kernel trace of C2 steps (gpurun_out/r3base)
set -e -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3base
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1
find $O -name "*stats*.csv"
