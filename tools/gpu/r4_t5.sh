#!/bin/bash
# round-4 check 5: the wave-pair scan forward (c1p): parity (c1 / c1p kernel
# tests, north-star width), then timing A/B c1 vs c1p, the fixed conv / C5 DP
# tests, the VALU cost microbenchmark and the c1 SQ PMC passes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t5
mkdir -p $O
cd $R
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_ops.py -k "c1" -x > $O/c1p.log 2>&1
rc=$?; echo "c1p tests rc=$rc"; tail -15 $O/c1p.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
timeout -k 10 300 python tools/gemm_k_sweep.py > $O/ksweep.jsonl 2> $O/ksweep.err || { tail $O/ksweep.err; exit 1; }
cat $O/ksweep.jsonl
timeout -k 10 300 $PT tests/test_gpu_c5_dp.py tests/test_gpu_ops.py -k "c5 or conv" > $O/tests.log 2>&1
echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 120 tools/ubench/valu_costs > $O/valu.txt 2>&1 || { tail $O/valu.txt; exit 1; }
cat $O/valu.txt
cd /tmp
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/fp32 -o p1 -- python3 $R/tools/scan_once.py fp32 > $O/fp32.log 2>&1 || { tail -5 $O/fp32.log; exit 1; }
ITERS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/fp32b -o p2 -- python3 $R/tools/scan_once.py fp32 > $O/fp32b.log 2>&1 || { tail -5 $O/fp32b.log; exit 1; }
python3 $R/tools/pmc_kernels.py $(find $O -name "*counter_collection.csv") --match scan > $O/scan_pmc.txt
cat $O/scan_pmc.txt
