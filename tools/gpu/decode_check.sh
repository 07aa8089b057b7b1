#!/bin/bash
# decode-step parity (module tests) + p50 of the engine (tools/decode_ab.py rowsonly)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_modules.py tests/test_gpu_configs.py > gpurun_out/t2.log 2>&1
tail -2 gpurun_out/t2.log
for i in 1 2; do DEC_STEPS=300 timeout -k 10 300 python -u tools/decode_ab.py rowsonly 2>&1 | grep -v amdgpu.ids; done
