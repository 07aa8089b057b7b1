#!/bin/bash
# round 6: the whole GPU suite, the style leg's bench numbers and kernel trace,
# then the default bench line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python tools/style_once.py > $O/style.json 2> $O/style.err || { tail $O/style.err; exit 1; }
cat $O/style.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/style -o style -- python3 $R/tools/style_once.py > $O/style.log 2>&1 || { tail -5 $O/style.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/c5_once.py > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
