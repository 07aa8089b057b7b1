#!/bin/bash
# scan forward: parity of every variant, then A/B timing
mkdir -p gpurun_out/s6
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k scan > gpurun_out/s6/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/s6/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/scan_ab.py 2>&1 | grep -v amdgpu.ids
