#!/bin/bash
# round-4 check 4: re-run the two fixed tests (conv override alias, C5 DP), the
# VALU issue-cost microbenchmark at 1/2/4/8 waves per SIMD, and the SQ PMC
# passes over the north-star scan forward (c1 kernel, fp32)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t4
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 170 --timeout-method thread tests/test_gpu_c5_dp.py tests/test_gpu_ops.py -k "c5 or conv" > $O/tests.log 2>&1
echo "tests rc=$?"; tail -5 $O/tests.log
timeout -k 10 120 tools/ubench/valu_costs > $O/valu.txt 2>&1 || { tail $O/valu.txt; exit 1; }
cat $O/valu.txt
cd /tmp
for dt in fp32; do
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/$dt -o p1 -- python3 $R/tools/scan_once.py $dt > $O/$dt.log 2>&1 || { tail -5 $O/$dt.log; exit 1; }
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/${dt}b -o p2 -- python3 $R/tools/scan_once.py $dt > $O/${dt}b.log 2>&1 || { tail -5 $O/${dt}b.log; exit 1; }
done
python3 $R/tools/pmc_kernels.py $(find $O -name "*counter_collection.csv") --match scan > $O/scan_pmc.txt
cat $O/scan_pmc.txt
