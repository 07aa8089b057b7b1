#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/valu_trans > gpurun_out/ubench.log 2>&1; rc=$?; echo "ubench rc=$rc"; cat gpurun_out/ubench.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_gpu_ops.py -m gpu -q -x > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -10
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_scan.py > gpurun_out/scan.log 2>&1; rc=$?; echo "scan rc=$rc"; grep -v amdgpu.ids gpurun_out/scan.log
