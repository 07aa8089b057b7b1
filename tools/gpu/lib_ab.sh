#!/bin/bash
# op A/B of two builds of libmtts.so: $ALT (path) vs the in-tree library; CMD = python script + args
set -e -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  echo "== in-tree"; timeout -k 10 300 python -u $CMD 2>&1 | grep -v amdgpu.ids
  echo "== $ALT"; MTTS_LIB=$ALT timeout -k 10 300 python -u $CMD 2>&1 | grep -v amdgpu.ids
done
