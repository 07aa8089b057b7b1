#!/bin/bash
# attention kernels: parity tests, then module tests
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_attention.py -x -q > gpurun_out/attn_tests.log 2>&1
rc=$?
tail -30 gpurun_out/attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_modules.py -x -q > gpurun_out/mod_tests.log 2>&1
rc=$?
tail -30 gpurun_out/mod_tests.log
exit $rc
