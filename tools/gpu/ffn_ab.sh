#!/bin/bash
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ffn
mkdir -p $O
timeout -k 10 400 python -u tools/ffn_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
