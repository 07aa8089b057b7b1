#!/bin/bash
# round-4 check 17: C2 scan backward per-kernel times and SQ issue counters
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t17
mkdir -p $O
cd /tmp
ITERS=10 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/tools/scan_bwd_once.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
ITERS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/scan_bwd_once.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
ITERS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 $R/tools/scan_bwd_once.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
cd $R
python tools/kstat_top.py $(find $O/kt -name "*kernel_stats.csv") 8
python tools/pmc_kernels.py $(find $O/p1 $O/p2 -name "*counter_collection.csv") --match scan
