#!/bin/bash
# hipBLASLt rates on the C2 GEMM shapes + a profiled C2-only bench run
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2b
mkdir -p $O
timeout -k 10 300 python tools/bench_gemm.py > $O/gemm.txt 2>&1 || { tail -20 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 -- python $R/bench.py --skip-extras --steps 5 --warmup 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -2 $O/bench.log
find $O/prof -name "*kernel_stats.csv" | head
