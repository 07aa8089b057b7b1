#!/bin/bash
# round 5: grouped / deferred weight gradients -- GEMM + engine tests, the
# decoder parity tests, then interleaved C2-step A/B: base / DEFER=0 / DEFER=1
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r5e}
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $PT tests/test_gpu_gemm.py tests/test_gpu_wgrad.py > $O/gemm.log 2>&1; rc=$?; tail -2 $O/gemm.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 $PT tests/test_gpu_ops.py -k "layernorm" tests/test_gpu_modules.py tests/test_gpu_configs.py tests/test_gpu_c5.py tests/test_gpu_dp.py > $O/mods.log 2>&1; rc=$?; tail -2 $O/mods.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  AB_ROOT=tools/ab/base timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  DEFER=0 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  DEFER=1 timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
done
cat $O/ab.txt
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c2 -o kt -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 5 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/kt.log; exit 1; }
find $GRAFT_REPO_ROOT/$O -name "*kernel_trace.csv" -size +20M -delete; find $GRAFT_REPO_ROOT/$O -name "*.db" -delete
echo done
