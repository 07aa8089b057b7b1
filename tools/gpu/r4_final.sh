#!/bin/bash
# round-4 closing pass: (1) rows past the ends with the previous library
# (row origins in the scalar offset) and with this tree; (2) the full -m gpu
# suite + smoke; (3) the default bench line; (4) kernel trace of the
# north-star scan forward (fp32).  Outputs: gpurun_out/fin/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fin
mkdir -p $O
cd $R
LIB=mamba-tts-project_amd/mtts/libmtts.so
cp $LIB /tmp/new_libmtts.so
cp tools/ab/base/$LIB $LIB
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_attention.py -k "rows_past" > $O/old.log 2>&1
echo "old lib rc=$?"; grep -E "passed|failed" $O/old.log | tail -2; grep -E "^FAILED" $O/old.log | head -20
cp /tmp/new_libmtts.so $LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo "GPU suite failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
ITERS=100 timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/scan -o trace_fp32 -- python3 $R/tools/scan_once.py fp32 > $O/scan.log 2>&1 || { tail -5 $O/scan.log; exit 1; }
grep "scan " $O/scan.log
find $O -name "*kernel_trace.csv" -size +20M -delete; find $O -name "*.db" -delete; du -sh $O
