#!/bin/bash
# Same-box A/B of this tree's libmtts.so against tools/ab/base (the previous
# commit's package: build it with `make` in a worktree of that commit and copy
# the .so + mtts/*.py there), the round-4 experiment recipe:
#   bash tools/gpu/ab_lib.sh <tool.py> [pytest -k expr]
# runs the parity subset first (tests/test_gpu_ops.py tests/test_gpu_configs.py
# tests/test_gpu_attention.py, optionally narrowed by -k), then three
# interleaved base / this-tree rounds of the timing tool (tools/scan_lib_ab.py,
# tools/attn_ab.py, ...; SWEEP / SHAPES pass through the environment).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
TOOL=$1; KARGS=(); [ -n "$2" ] && KARGS=(-k "$2")
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_attention.py -x "${KARGS[@]}" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  echo "== base" >> $O/ab.txt; AB_ROOT=tools/ab/base timeout -k 10 300 python $TOOL >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== new" >> $O/ab.txt; timeout -k 10 300 python $TOOL >> $O/ab.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/ab.txt
