#!/bin/bash
# SQ counters for the wide scan forward (bf16 north-star), normal and compute-only builds
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM"
timeout -k 10 200 rocprofv3 --pmc $C1 --output-format csv -d $R/gpurun_out/pmc3 -o w1 -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/pmc3/w1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc $C2 --output-format csv -d $R/gpurun_out/pmc3 -o w2 -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/pmc3/w2.log 2>&1 || exit 1
MTTS_LIB=$R/tools/diag/libmtts_nomem.so timeout -k 10 200 rocprofv3 --pmc $C1 --output-format csv -d $R/gpurun_out/pmc3 -o n1 -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/pmc3/n1.log 2>&1 || exit 1
timeout -k 10 100 python3 tools/scan_once.py bf16
MTTS_LIB=$R/tools/diag/libmtts_nomem.so timeout -k 10 100 python3 tools/scan_once.py bf16
