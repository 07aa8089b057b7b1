#!/bin/bash
# round 5: parity subset for the LN / FiLM / bias-slot change, then an
# interleaved C2-step A/B against tools/ab/base (3 rounds)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r5c}
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_ops.py -k "layernorm or conv" > $O/ops.log 2>&1; rc=$?; tail -2 $O/ops.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 $PT tests/test_gpu_modules.py tests/test_gpu_configs.py tests/test_gpu_style.py ${EXTRA_TESTS} > $O/mods.log 2>&1; rc=$?; tail -2 $O/mods.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  AB_ROOT=tools/ab/base timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
  timeout -k 10 200 python tools/c2_ab.py 2>/dev/null >> $O/ab.txt || exit 1
done
cat $O/ab.txt
