#!/bin/bash
# convgemm NN data gradient: kernel / text / C5 tests, per-shape timings, text leg profile
OUT=gpurun_out/r5s; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_convgemm.py \
  tests/test_gpu_text.py tests/test_gpu_c5.py tests/test_gpu_c5_dp.py > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/convgemm_bench.py > $OUT/bench.txt 2>&1 && \
timeout -k 10 200 python -u tools/text_prof.py > $OUT/text_prof.txt 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -v amdgpu.ids $OUT/bench.txt; head -14 $OUT/text_prof.txt; exit $rc
