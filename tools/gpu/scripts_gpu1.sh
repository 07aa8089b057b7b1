#!/bin/bash
# GPU session script: tests, smoke, bench (each step time-limited)
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --decode-steps 200 --cpu-budget 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -12 gpurun_out/bench.log
