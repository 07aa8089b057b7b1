#!/bin/bash
# conv parity tests, then tiled vs untiled conv kernels at the C2 shape
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/conv
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "conv" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python -u tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
