#!/bin/bash
# round-4 check 12: the 2-wave-block pair scan forward (c1p): parity, c1 vs
# c1p timing, SQ PMC of c1p (fp32)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t12
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "c1" -x > $O/c1p.log 2>&1
rc=$?; echo "c1p tests rc=$rc"; tail -3 $O/c1p.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/scan_lib_ab.py >> $O/ab.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
cd /tmp
export SCAN_PATH=4 ITERS=2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/scan_once.py fp32 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
grep "scan " $O/p1.log
