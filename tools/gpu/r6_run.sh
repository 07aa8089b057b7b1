#!/bin/bash
# round-6 combined GPU pass: targeted parity tests, same-box attention A/B
# against tools/ab/base, then the default bench line.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_dropout.py tests/test_gpu_attention.py tests/test_gpu_c5.py tests/test_gpu_style.py \
  tests/test_gpu_text.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
if [ "${AB:-1}" = "1" ]; then
  for i in 1 2 3; do
    echo "== base" >> $O/attn_ab.txt; AB_ROOT=tools/ab/base SHAPES=C5m,C5 timeout -k 10 300 python tools/attn_ab.py >> $O/attn_ab.txt 2>>$O/err || { tail $O/err; exit 1; }
    echo "== new" >> $O/attn_ab.txt; SHAPES=C5m,C5 timeout -k 10 300 python tools/attn_ab.py >> $O/attn_ab.txt 2>>$O/err || { tail $O/err; exit 1; }
  done
  cat $O/attn_ab.txt
fi
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
