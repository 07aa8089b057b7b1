#!/bin/bash
# PMC passes over one C2 training step (plus 2 warmup steps): SQ issue/stall
# breakdown and MFMA activity per kernel
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_c2
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|GRBM_[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt || true
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p1 -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 1 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p2 -o p2 -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 1 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O -name "*.csv" | head
