#!/bin/bash
# round 6: K/V batching glue fix -- decoder / DP / C5 parity, then the bench line and a C2 step trace
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6kv
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread \
  tests/test_gpu_kvall.py tests/test_gpu_wgrad.py tests/test_gpu_c5.py tests/test_gpu_c5_dp.py tests/test_gpu_dp.py \
  tests/test_gpu_modules.py tests/test_gpu_configs.py tests/test_gpu_attention.py tests/test_gpu_style.py tests/test_gpu_dropout.py tests/test_gpu_text.py "tests/test_gpu_ops.py::test_tn_fused_column_sums" "tests/test_gpu_ops.py::test_wgrad_split_k_matches_fp64" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o kt -- python3 $R/tools/gemm_step_ab.py hip 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
