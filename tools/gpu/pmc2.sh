#!/bin/bash
# SQ counters for the north-star scan forward (bf16); counter list saved for reference
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc2/counters.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" gpurun_out/pmc2/counters.txt | sort -u > gpurun_out/pmc2/sq_names.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc2 -o sq1 -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/pmc2/sq1.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/pmc2/sq1.log
ls gpurun_out/pmc2
