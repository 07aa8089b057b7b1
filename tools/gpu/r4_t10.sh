#!/bin/bash
# round-4 check 10: fused split-K reduction in the TN GEMM: GEMM parity
# (fused == separate launch, bit-exact), C2 routing / decoder tests, TN K-sweep
# and the C2 step A/B (separate reduce launch vs fused)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t10
mkdir -p $O
cd $R
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_gemm.py -x -k "fused_split" > $O/fused.log 2>&1
rc=$?; echo "fused test rc=$rc"; tail -4 $O/fused.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 700 $PT tests/test_gpu_gemm.py tests/test_gpu_configs.py tests/test_gpu_dp.py tests/test_gpu_c5_dp.py tests/test_gpu_attention.py -x > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/gemm_k_sweep.py > $O/ksweep.jsonl 2> $O/ksweep.err || { tail $O/ksweep.err; exit 1; }
grep '"tn"' $O/ksweep.jsonl
timeout -k 10 400 python tools/gemm_step_ab.py ovr gemm_split 1 > $O/step_ab.log 2>&1 || { tail $O/step_ab.log; exit 1; }
cat $O/step_ab.log
SHAPES=C5m timeout -k 10 200 python tools/attn_ab.py > $O/attn.log 2>&1 || { tail $O/attn.log; exit 1; }
cat $O/attn.log
