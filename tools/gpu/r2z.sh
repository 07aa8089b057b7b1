#!/bin/bash
# full GPU suite, smoke, default bench line
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/suite.log 2>&1
tail -3 gpurun_out/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err
tail -1 gpurun_out/bench.log
