#!/bin/bash
# full -m gpu suite, then the C5 train.py step twice
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fullc5
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  timeout -k 10 300 python -u -c "
import json,sys; sys.path[:0]=['.','mamba-tts-project_amd']
import bench; print(json.dumps(bench.c5_step_bench(0,1,'cuda',steps=5)))" > $O/c5_$i.json 2> $O/c5_$i.err || { tail -20 $O/c5_$i.err; exit 1; }
  echo "c5 $(grep -o '"ms_per_step": [0-9.]*' $O/c5_$i.json)"
done
