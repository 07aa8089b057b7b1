#!/bin/bash
# full -m gpu suite, smoke, default bench line (gpurun_out/final)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
