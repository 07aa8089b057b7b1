#!/bin/bash
# gemm-related GPU tests, then in-process C2 step A/B of the GEMM routing
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/step
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_configs.py tests/test_gpu_c5.py tests/test_gpu_attention.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/gemm_step_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
