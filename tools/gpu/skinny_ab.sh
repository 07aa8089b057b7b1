#!/bin/bash
# skinny GEMM tests + the Mamba / decoder tests that route through them, then the A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/skinny
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_configs.py tests/test_gpu_c5.py tests/test_gpu_modules.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 400 python -u tools/skinny_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
