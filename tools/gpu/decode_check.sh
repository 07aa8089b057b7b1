#!/bin/bash
# decode parity tests (module goldens, C4 4096-step test), then the C4 decode latency twice
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dec
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_modules.py tests/test_gpu_configs.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  timeout -k 10 300 python -u -c "
import json,sys; sys.path[:0]=['.','mamba-tts-project_amd']
import bench; print(json.dumps(bench.decode_bench(2000)))" > $O/d_$i.json 2> $O/d_$i.err || { tail -20 $O/d_$i.err; exit 1; }
  cat $O/d_$i.json
done
