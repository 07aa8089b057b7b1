#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_modules.py > gpurun_out/diag.log 2>&1; rc=$?; echo "diag rc=$rc"; cat gpurun_out/diag.log | grep -v amdgpu.ids
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_gpu_ops.py -m gpu -q > gpurun_out/pytest_ops.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest_ops.log | tail -40
