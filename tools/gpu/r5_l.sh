#!/bin/bash
# measurement pass for the C5 per-tensor bounds (the tests fail until the bounds are filled in)
OUT=gpurun_out/r5l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -s -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py::test_c5_train_shape_two_layer_decoder_bf16 \
  tests/test_gpu_c5.py::test_c5_train_py_width_bf16_one_step_vs_oracle > $OUT/c5.log 2>&1
grep "measured errors" $OUT/c5.log; tail -3 $OUT/c5.log; exit 0
