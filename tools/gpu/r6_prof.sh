#!/bin/bash
# round 6: attention A/B (dQ LDS-DMA vs base), then kernel traces of the
# style leg and of the C5 step
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6p
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_dropout.py tests/test_gpu_ops.py -k 'layernorm or ln_ or attention or dropout' > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
for i in; do
  echo "== base" >> $O/attn_ab.txt; AB_ROOT=tools/ab/base SHAPES=C5m timeout -k 10 300 python tools/attn_ab.py >> $O/attn_ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  echo "== new" >> $O/attn_ab.txt; SHAPES=C5m timeout -k 10 300 python tools/attn_ab.py >> $O/attn_ab.txt 2>>$O/err || { tail $O/err; exit 1; }
done
cat $O/attn_ab.txt
timeout -k 10 120 python tools/bench_ln.py > $O/ln.txt 2>&1 || { tail $O/ln.txt; exit 1; }
cat $O/ln.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/style -o style -- python3 $R/tools/style_once.py > $O/style.log 2>&1 || { tail -5 $O/style.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/c5_once.py > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
find $O -name "*kernel_stats.csv" | head
