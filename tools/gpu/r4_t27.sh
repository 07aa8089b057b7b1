#!/bin/bash
# round-4 check 27: scan carry kernel back on DPP broadcasts (31.7 KiB LDS:
# 5 blocks per CU, every carry block of K = 6 resident at once): parity, then
# segment sweep for this tree and the base
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t27
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "scan or bwd" -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  AB_ROOT=tools/ab/base SWEEP="scan_bwd_segs=4,5,6,8" timeout -k 10 200 python tools/scan_lib_ab.py >> $O/sweep.jsonl 2>>$O/err || { tail $O/err; exit 1; }
  SWEEP="scan_bwd_segs=4,5,6,8" timeout -k 10 200 python tools/scan_lib_ab.py >> $O/sweep.jsonl 2>>$O/err || { tail $O/err; exit 1; }
done
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['pkg'][:12], {k[-6:]:v for k,v in d.items() if 'bwd' in k})
"
