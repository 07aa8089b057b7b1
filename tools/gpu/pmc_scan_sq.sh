#!/bin/bash
# SQ issue / stall PMC pass over the north-star scan forward (c1, fp32 and bf16)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_scan
mkdir -p $O
cd /tmp
for dt in fp32 bf16; do
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/$dt -o p1 -- python3 $GRAFT_REPO_ROOT/tools/scan_once.py $dt > $O/$dt.log 2>&1 || { tail -5 $O/$dt.log; exit 1; }
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/${dt}b -o p2 -- python3 $GRAFT_REPO_ROOT/tools/scan_once.py $dt > $O/${dt}b.log 2>&1 || { tail -5 $O/${dt}b.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
