#!/bin/bash
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for dt in bf16 fp32; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc -o trace_$dt -- python3 $R/tools/scan_once.py $dt > $R/gpurun_out/pmc/trace_$dt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc -o fetch_$dt -- python3 $R/tools/scan_once.py $dt > $R/gpurun_out/pmc/fetch_$dt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc -o write_$dt -- python3 $R/tools/scan_once.py $dt > $R/gpurun_out/pmc/write_$dt.log 2>&1 || exit 1
done
ls $R/gpurun_out/pmc
