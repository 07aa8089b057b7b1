#!/bin/bash
# round-4 check 6: SQ PMC passes over the wave-pair scan forward (c1p, fp32)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t6
mkdir -p $O
cd /tmp
export SCAN_PATH=4 ITERS=2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/scan_once.py fp32 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 $R/tools/scan_once.py fp32 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/p3 -o p3 -- python3 $R/tools/scan_once.py fp32 > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 0; }
grep scan $O/p1.log
