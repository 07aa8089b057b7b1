#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/wgrad.log 2>&1; rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/wgrad.log
