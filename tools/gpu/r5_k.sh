#!/bin/bash
# four-wave NT tile: GEMM tests, then the same-process tile A/B
set -o pipefail
OUT=gpurun_out/r5k; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "four_wave or every_kernel or nt_" > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_tile_ab.py 3 > $OUT/ab.txt 2>&1
rc=$?; tail -3 $OUT/tests.log; cat $OUT/ab.txt; exit $rc
