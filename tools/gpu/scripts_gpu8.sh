#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --decode-steps 0 --cpu-budget 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep "\[bench\]" gpurun_out/bench.log; tail -3 gpurun_out/bench.log | grep -v "^{"
