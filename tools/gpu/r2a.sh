#!/bin/bash
# round 2, first GPU pass: new config/contract tests, the whole -m gpu suite,
# a 2-rank gloo rehearsal of the bench's DP launch on the one GPU, the bench line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2a
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_configs.py tests/test_gpu_dp.py -m gpu > $O/new_tests.log 2>&1; rc=$?
echo "new tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/new_tests.log | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 1200 $PT tests -m gpu --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_dp.py > $O/pytest.log 2>&1; rc2=$?
echo "full suite rc=$rc2"; tail -3 $O/pytest.log
[ $rc2 -ne 0 ] && [ $rc2 -ne 1 ] && exit $rc2
MTTS_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 > $O/bench_g2.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 1; }
cat $O/bench_g2.json
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
