#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_scan.py > gpurun_out/scan.log 2>&1; rc=$?; echo "scan rc=$rc"; grep -v amdgpu.ids gpurun_out/scan.log
