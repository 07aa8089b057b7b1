#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --decode-steps 200 --cpu-budget 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep "\[bench\]" gpurun_out/bench.log; tail -1 gpurun_out/bench.log
