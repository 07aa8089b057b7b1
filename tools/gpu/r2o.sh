#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2o
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_ops.py -m gpu -k "conv" > $O/conv_tests.log 2>&1; rc=$?
tail -2 $O/conv_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 60 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | sed 's/^/new: /'
MTTS_LIB=$GRAFT_REPO_ROOT/mamba-tts-project_amd/mtts/libmtts_convold.so timeout -k 10 60 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | sed 's/^/old: /'
done
