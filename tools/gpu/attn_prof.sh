#!/bin/bash
# attention parity tests, then a kernel-trace profile of tools/attn_ab.py (SHAPES env)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attnprof
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_attention.py tests/test_gpu_c5.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
cd /tmp && export TMPDIR=/tmp
SHAPES=${SHAPES:-C5m,C5} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/attn_ab.py > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
grep -E "fwd|bwd" $O/run.log
