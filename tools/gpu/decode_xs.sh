#!/bin/bash
# fused x_proj + state update: op + decode parity tests, then the decode-step A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dxs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "xproj or state" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_modules.py tests/test_gpu_configs.py > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
DEC_STEPS=200 timeout -k 10 300 python -u tools/decode_ab.py xs 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
