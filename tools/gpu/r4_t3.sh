#!/bin/bash
# round-4 check 3: C5 DP test alone (diagnostic), the GPU suite without it,
# scan A/B (tools/ab/base = round-3 HEAD package vs this tree), default bench,
# C2-step kernel trace, decode-step kernel trace, attention SQ PMC at C5.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t3
mkdir -p $O
cd $R
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 python -u -m pytest -q -s --timeout 170 --timeout-method thread tests/test_gpu_c5_dp.py > $O/c5dp.log 2>&1
echo "c5dp rc=$?"; tail -30 $O/c5dp.log
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu --deselect tests/test_gpu_c5_dp.py::test_c5_train_step_dp_world2_matches_single_process_mean_loss > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2 3; do
  AB_ROOT=$R/tools/ab/base timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  echo "ab round $i"
done
cat $O/ab.jsonl
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o kt -- python3 $R/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo "c2 trace done"
DEC_STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 $R/tools/decode_ab.py rowsonly > $O/dec.log 2>&1 || { tail -20 $O/dec.log; exit 1; }
echo "decode trace done"
export SHAPES=C5m
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/attn -o p1 -- python3 $R/tools/attn_ab.py > $O/attn_p1.log 2>&1 || { tail -5 $O/attn_p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/attn -o p2 -- python3 $R/tools/attn_ab.py > $O/attn_p2.log 2>&1 || { tail -5 $O/attn_p2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d $O/attn -o p3 -- python3 $R/tools/attn_ab.py > $O/attn_p3.log 2>&1 || { tail -5 $O/attn_p3.log; exit 1; }
python3 $R/tools/pmc_kernels.py $(find $O/attn -name "*counter_collection.csv") --match attn > $O/attn_summary.txt
cat $O/attn_summary.txt
find $O -name "*.db" -delete; find $O -name "*kernel_trace.csv" -size +30M -delete; du -sh $O
