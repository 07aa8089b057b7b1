#!/bin/bash
# round-4 check 9: attention (dK/dV slice buffer loads) parity + timing, then
# the full GPU suite and the default bench line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t9
mkdir -p $O
cd $R
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_attention.py tests/test_gpu_c5.py -x > $O/attn_tests.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -3 $O/attn_tests.log
[ $rc -eq 0 ] || exit 1
SHAPES=C5m timeout -k 10 200 python tools/attn_ab.py > $O/attn.log 2>&1 || { tail $O/attn.log; exit 1; }
cat $O/attn.log
timeout -k 10 900 $PT tests -m gpu > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 $O/suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('roofline', d['roofline']['ms'], d['roofline']['frac'], 'bf16', d['roofline_bf16']['ms'], 'c5', d['c5_step']['ms_per_step'], 'decode', d['decode']['p50_ms'], 'te', d['text_encoder']['fwd_bwd_ms'])"
