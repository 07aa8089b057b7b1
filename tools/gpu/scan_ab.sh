#!/bin/bash
# scan forward parity tests, then north-star A/B of the c1 variants
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/scan
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "scan" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "north or c2_shape_scan or scan" > $O/test2.log 2>&1 || { tail -30 $O/test2.log; exit 1; }
tail -1 $O/test2.log
timeout -k 10 300 python -u tools/scan_ab.py xl c1big 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
