#!/bin/bash
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --skip-extras > $R/gpurun_out/prof1/bench.log 2>&1; rc=$?; echo "prof rc=$rc"
find $R/gpurun_out/prof1 -name "*stats*" | head
