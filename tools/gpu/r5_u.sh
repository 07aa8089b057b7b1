#!/bin/bash
# grouped-wgrad fallback: wgrad / gemm / C5 tests, C5 step trace, C5 + C2 bench legs
OUT=gpurun_out/r5u; mkdir -p $OUT/c5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad.py \
  tests/test_gpu_gemm.py tests/test_gpu_c5.py > $OUT/tests.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o c5 -- python3 tools/c5_once.py > $OUT/c5/c5.log 2>&1 && \
timeout -k 10 300 python -u tools/c2_ab.py > $OUT/ab.txt 2>&1
rc=$?; tail -2 $OUT/tests.log; tail -4 $OUT/c5/c5.log; tail -4 $OUT/ab.txt; find $OUT -name "*kernel_trace.csv" -delete; exit $rc
