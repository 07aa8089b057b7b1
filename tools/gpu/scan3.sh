#!/bin/bash
# scan kernels: parity, then north-star timing normal vs compute-only diag build, C2 bench
mkdir -p gpurun_out/scan3
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_modules.py -x -q > gpurun_out/scan3/tests.log 2>&1; rc=$?
tail -5 gpurun_out/scan3/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/scan_once.py bf16 || exit 1
MTTS_LIB=$PWD/tools/diag/libmtts_nomem.so timeout -k 10 100 python tools/scan_once.py bf16 || exit 1
timeout -k 10 300 python tools/bench_scan.py quick > gpurun_out/scan3/bench_scan.log 2>&1 || exit 1
cat gpurun_out/scan3/bench_scan.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --decode-steps 0 --cpu-budget 0 > gpurun_out/scan3/bench.log 2>&1 || exit 1
grep "\[bench\]" gpurun_out/scan3/bench.log
