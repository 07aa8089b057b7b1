#!/bin/bash
# full GPU suite + C2 bench (no extras)
mkdir -p gpurun_out/s9
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s9/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/s9/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --skip-extras 2> gpurun_out/s9/bench.err | tee gpurun_out/s9/bench.json
grep "\[bench\]" gpurun_out/s9/bench.err
