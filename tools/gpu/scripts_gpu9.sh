#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -m gpu -q -x > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
for segs in 2 4 8; do MTTS_SCAN_BWD_SEGS=$segs timeout -k 10 120 python tools/bench_scan.py quick 2>&1 | grep bwd | sed "s/^/segs=$segs /"; done
