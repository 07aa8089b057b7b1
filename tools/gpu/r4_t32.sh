#!/bin/bash
# round-4 check 32: call sites of the torch glue kernels in one C2 step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/t32
cd $R
timeout -k 10 300 python tools/glue_sources.py > gpurun_out/t32/glue.txt 2>&1 || { tail -20 gpurun_out/t32/glue.txt; exit 1; }
cat gpurun_out/t32/glue.txt
