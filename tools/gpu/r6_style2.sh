#!/bin/bash
# round 6: style-pipeline tests + the style leg's numbers and kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6t
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -q -m gpu -x --timeout 200 --timeout-method thread \
  tests/test_gpu_dropout.py tests/test_gpu_style.py tests/test_gpu_modules.py tests/test_gpu_c5.py tests/test_gpu_text.py tests/test_gpu_convgemm.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python tools/style_once.py > $O/style.json 2> $O/style.err || { tail $O/style.err; exit 1; }
cat $O/style.json
timeout -k 10 300 python -c "import sys, json; sys.path[:0] = ['.', 'mamba-tts-project_amd']; import bench; print(json.dumps(bench.text_bench()))" > $O/text.json 2> $O/text.err || { tail $O/text.err; exit 1; }
cat $O/text.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/style -o style -- python3 $R/tools/style_once.py > $O/style.log 2>&1 || { tail -5 $O/style.log; exit 1; }
