#!/bin/bash
# round 5, call B: baseline of this round -- default bench line, C2-step
# kernel trace (rocprofv3 --kernel-trace --stats over 2 warmup + 5 steps),
# and the glue-kernel attribution of one C2 step
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5b}
mkdir -p $O/c2
cd $R
timeout -k 10 300 python tools/glue_sources.py > $O/glue.txt 2>&1 || { tail -20 $O/glue.txt; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o kt -- python3 $R/tools/gemm_step_ab.py hip 5 > $O/c2/kt.log 2>&1 || { tail -5 $O/c2/kt.log; exit 1; }
find $O -name "*kernel_trace.csv" -size +20M -delete; find $O -name "*.db" -delete
python3 $R/tools/kstat_top.py $(find $O/c2 -name "*kernel_stats.csv" | head -1) 45 > $O/c2_top.txt; head -5 $O/c2_top.txt
