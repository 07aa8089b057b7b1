#!/bin/bash
# round 6: LayerNorm backward (two raw rows in flight) -- parity, then same-box A/B of tools/bench_ln.py
# against tools/ab/base (one raw row ahead), three interleaved rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ln
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread \
  tests/test_gpu_ops.py -k "layernorm or ln_ or gemm_rows_ln" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_text.py tests/test_gpu_style.py tests/test_gpu_modules.py tests/test_gpu_c5.py > $O/tests2.log 2>&1
rc=$?; echo "tests2 rc=$rc"; tail -2 $O/tests2.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests2.log | head -30; exit 1; }
for i in 1 2 3; do
  echo "== base" >> $O/ab.txt; AB_ROOT=tools/ab/base timeout -k 10 120 python tools/bench_ln.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== new" >> $O/ab.txt; timeout -k 10 120 python tools/bench_ln.py >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/ab.txt
