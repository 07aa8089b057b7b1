#!/bin/bash
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tune/tunableop_results%d.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20
( timeout -k 10 500 python tools/bench_gemm.py > gpurun_out/tune/tuned_first.log 2>&1 ) ; echo "rc=$?"
tail -12 gpurun_out/tune/tuned_first.log
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 200 python tools/bench_gemm.py 2>&1 | grep -v amdgpu.ids
