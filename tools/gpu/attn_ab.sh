#!/bin/bash
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/attn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_attention.py tests/test_gpu_text.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/attn_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
