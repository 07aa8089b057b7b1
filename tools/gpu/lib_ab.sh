#!/bin/bash
# A/B of a diag library build against the default one, alternated:
#   tools/gpu/lib_ab.sh NAME "<python command>" [rounds]
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq ${3:-3}); do
  echo "== round $i base"
  timeout -k 10 150 $2
  echo "== round $i $1"
  MTTS_LIB=$GRAFT_REPO_ROOT/mamba-tts-project_amd/mtts/libmtts_$1.so timeout -k 10 150 $2
done
