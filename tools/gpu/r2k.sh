#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2k
mkdir -p $O
L=$GRAFT_REPO_ROOT/mamba-tts-project_amd/mtts
for v in base cnodma cfix cnost cfixnost; do
  if [ $v = base ]; then lib=$L/libmtts.so; else lib=$L/libmtts_$v.so; fi
  MTTS_LIB=$lib timeout -k 10 120 python tools/scan_ab.py xl > $O/$v.txt 2>&1 || { cat $O/$v.txt; exit 1; }
  echo "$v: $(grep -v amdgpu.ids $O/$v.txt | tr '\n' ' ')"
done
