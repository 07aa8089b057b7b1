#!/bin/bash
# SQ / MFMA PMC passes over the fp32 conv GEMM (tools/convgemm_once.py). Outputs: gpurun_out/cgpmc/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cgpmc
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p1 -- python3 $R/tools/convgemm_once.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- python3 $R/tools/convgemm_once.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- python3 $R/tools/convgemm_once.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 $R/tools/pmc_kernels.py $O/p1_counter_collection.csv $O/p2_counter_collection.csv > $O/summary.txt 2>&1; cat $O/summary.txt | cut -c1-400
