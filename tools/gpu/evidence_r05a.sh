#!/bin/bash
# Round-5 evidence, part 1: the full -m gpu suite + smoke.  Outputs: gpurun_out/ev5/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${EVDIR:-ev5}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
