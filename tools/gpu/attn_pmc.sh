#!/bin/bash
# PMC passes over tools/attn_ab.py (SHAPES env) for the attention kernels
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attnpmc
mkdir -p $O
export SHAPES=${SHAPES:-C5m}
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O -o p1 -- python3 $R/tools/attn_ab.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- python3 $R/tools/attn_ab.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d $O -o p3 -- python3 $R/tools/attn_ab.py > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python3 $R/tools/pmc_kernels.py $(find $O -name "*counter_collection.csv") --match attn > $O/summary.txt
cat $O/summary.txt
