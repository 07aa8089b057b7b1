#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_modules.py -m gpu -q > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -12
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "
import sys; sys.argv=['bench']; import bench, json
print(json.dumps(bench.decode_bench(300)))
" 2>&1 | grep -v amdgpu
