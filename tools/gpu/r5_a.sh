#!/bin/bash
# round 5, call A: conv buffer-addressed forward + poisoned-row tests, ADVICE
# fixes (shim mixer test, decode reset), conv A/B vs tools/ab/base, glue sources
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "conv or rows_past or scan_c1" > $O/ops.log 2>&1; rc=$?; tail -3 $O/ops.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_modules.py \
  > $O/modules.log 2>&1; rc=$?; tail -3 $O/modules.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  echo "== base" >> $O/conv_ab.txt; AB_ROOT=tools/ab/base timeout -k 10 120 python tools/bench_conv.py 2>/dev/null >> $O/conv_ab.txt || exit 1
  echo "== new" >> $O/conv_ab.txt; timeout -k 10 120 python tools/bench_conv.py 2>/dev/null >> $O/conv_ab.txt || exit 1
done
cat $O/conv_ab.txt
timeout -k 10 200 python tools/dbg/conv_dbg.py > $O/conv_dbg_after.txt 2>&1; timeout -k 10 300 python tools/glue_sources.py > $O/glue.txt 2>&1; echo glue rc=$?
