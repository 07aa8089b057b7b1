#!/bin/bash
# round-4 check 34: rows past the ends (NaN-poisoned, sentinel outputs) with
# the previous library (row origins in the scalar offset) and with this tree
# (row origins in the vector offset): does the buffer range check cover the
# scalar offset?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t34
mkdir -p $O
cd $R
LIB=mamba-tts-project_amd/mtts/libmtts.so
cp $LIB /tmp/new_libmtts.so
cp tools/ab/base/$LIB $LIB
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_attention.py -k "rows_past" > $O/old.log 2>&1
echo "old lib rc=$?"; grep -E "passed|failed" $O/old.log | tail -3; grep -E "^FAILED" $O/old.log | head -20
cp /tmp/new_libmtts.so $LIB
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_attention.py -k "rows_past" > $O/new.log 2>&1
echo "new lib rc=$?"; grep -E "passed|failed" $O/new.log | tail -3; grep -E "^FAILED" $O/new.log | head -20
