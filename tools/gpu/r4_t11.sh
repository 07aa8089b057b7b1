#!/bin/bash
# round-4 check 11: fused split-K with write-through slab stores: parity,
# TN timings, C2 step A/B (separate reduce launch vs fused)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t11
mkdir -p $O
cd $R
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_gemm.py -x -k "fused_split or tn" > $O/fused.log 2>&1
rc=$?; echo "fused test rc=$rc"; tail -3 $O/fused.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/gemm_k_sweep.py > $O/ksweep.jsonl 2> $O/ksweep.err || { tail $O/ksweep.err; exit 1; }
grep '"tn"' $O/ksweep.jsonl | grep -v '"splits": 1,'
timeout -k 10 400 python tools/gemm_step_ab.py ovr gemm_split 1 > $O/step_ab.log 2>&1 || { tail $O/step_ab.log; exit 1; }
cat $O/step_ab.log
