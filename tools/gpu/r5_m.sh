#!/bin/bash
# C5 tests with the measured bounds; text-encoder leg profile
OUT=gpurun_out/r5m; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py::test_c5_train_shape_two_layer_decoder_bf16 tests/test_gpu_c5.py > $OUT/c5.log 2>&1 && \
timeout -k 10 200 python -u tools/text_prof.py > $OUT/text_prof.txt 2>&1
rc=$?; tail -3 $OUT/c5.log; cat $OUT/text_prof.txt; exit $rc
