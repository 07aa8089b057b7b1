#!/bin/bash
# full GPU test suite + default bench line
mkdir -p gpurun_out/s1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/s1/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err; rc=$?; echo "bench rc=$rc"; grep "\[bench\]" gpurun_out/s1/bench.err; cat gpurun_out/s1/bench.json
exit $rc
