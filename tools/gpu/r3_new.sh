#!/bin/bash
# round-3 new coverage first (C5 harness, C4 4096-step decode, token check), then the full suite
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3new
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_c5.py \
  "tests/test_gpu_configs.py::test_c4_decode_4096_steps_vs_teacher_forced" \
  "tests/test_gpu_modules.py::test_decode_engine_out_of_range_token_raises" > $O/new.log 2>&1
grep -E "PASS|FAIL|C4 " $O/new.log | tail -12
[ -n "$NEW_ONLY" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
[ -n "$NEW_ONLY" ] || tail -1 $O/suite.log
