#!/bin/bash
# fused decode q projection: kernel + engine tests, C4 4096-step test, graph-replay A/B
OUT=gpurun_out/r5r; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_attention.py -k "qproj or decode" tests/test_gpu_modules.py \
  tests/test_gpu_configs.py::test_c4_decode_4096_steps_vs_teacher_forced > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/decode_ab.py opt:fuse_q > $OUT/ab.txt 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -v amdgpu.ids $OUT/ab.txt | tail -8; exit $rc
