#!/bin/bash
# round 5: full -m gpu suite + smoke on the current library, then the C2-step
# A/B (base / DEFER=0 / DEFER=1, 3 interleaved rounds)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r5f}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
  tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  grep -i smoke $O/smoke.log | tail -2
fi
for i in 1 2 3; do
  AB_ROOT=tools/ab/base timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  DEFER=0 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  DEFER=1 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
done
cat $O/ab.txt
