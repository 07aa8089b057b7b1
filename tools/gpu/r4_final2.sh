#!/bin/bash
# round-4 closing pass 2 (final library): full -m gpu suite + smoke, bench line,
# north-star scan kernel trace.  Outputs: gpurun_out/fin2/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fin2
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo "GPU suite failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
ITERS=100 timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/scan -o trace_fp32 -- python3 $R/tools/scan_once.py fp32 > $O/scan.log 2>&1 || { tail -5 $O/scan.log; exit 1; }
grep "scan " $O/scan.log
find $O -name "*kernel_trace.csv" -size +20M -delete; find $O -name "*.db" -delete; du -sh $O
