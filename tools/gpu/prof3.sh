#!/bin/bash
# full GPU test suite, bench (no extras), profiled C2 step
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest.log | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --skip-extras > gpurun_out/prof3/bench_plain.log 2>&1 || exit 1
grep "\[bench\]" gpurun_out/prof3/bench_plain.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --skip-extras > $R/gpurun_out/prof3/bench.log 2>&1; rc=$?; echo "prof rc=$rc"; grep "\[bench\]" $R/gpurun_out/prof3/bench.log
