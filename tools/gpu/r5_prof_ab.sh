#!/bin/bash
# kernel traces of the C2 step for tools/ab/base and this tree (tools/c2_ab.py: 2 + 15 steps each)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5p}
mkdir -p $O
cd /tmp
AB_ROOT=$R/tools/ab/base timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o kt -- python3 $R/tools/c2_ab.py > $O/base.log 2>&1 || { tail -5 $O/base.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o kt -- python3 $R/tools/c2_ab.py > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete
python3 $R/tools/kstat_diff.py $(find $O/base -name "*kernel_stats.csv") $(find $O/new -name "*kernel_stats.csv") 17 45
