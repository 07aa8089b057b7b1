#!/bin/bash
# direct fp32 convolutions: kernel tests, text-encoder parity, C5 tests, text leg profile
OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_convgemm.py \
  tests/test_gpu_text.py tests/test_gpu_c5.py > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/text_prof.py > $OUT/text_prof.txt 2>&1
rc=$?; tail -15 $OUT/tests.log; head -30 $OUT/text_prof.txt; exit $rc
