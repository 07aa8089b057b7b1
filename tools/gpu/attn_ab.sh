#!/bin/bash
# attention parity (incl. C5 long-KV), then the C5 step with the double-buffered
# bf16 forward on/off, alternating processes
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/attnab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_attention.py tests/test_gpu_c5.py} > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for db in 0 1 0 1; do
  MTTS_ATTN_FWD_DB=$db timeout -k 10 300 python -u -c "
import json,os,sys; sys.path[:0]=['.','mamba-tts-project_amd']
import bench; r=bench.c5_step_bench(0,1,'cuda',steps=5); print(json.dumps(r))" > $O/c5_$db.json 2> $O/c5_$db.err || { tail -20 $O/c5_$db.err; exit 1; }
  echo "db=$db $(grep -o '"ms_per_step": [0-9.]*' $O/c5_$db.json)"
done
