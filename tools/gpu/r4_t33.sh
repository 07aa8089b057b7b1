#!/bin/bash
# round-4 check 33: scan forward rows past L (NaN-poisoned inputs, sentinel
# output rows) for every forward path; then the glue-kernel call sites
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t33
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_attention.py -k "rows_past" > $O/tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|Error|assert" $O/tests.log | head -30
timeout -k 10 300 python tools/glue_sources.py > $O/glue.txt 2>&1 || { tail -20 $O/glue.txt; exit 1; }
cat $O/glue.txt
