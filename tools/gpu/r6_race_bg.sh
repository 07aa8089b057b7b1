#!/bin/bash
# round 6: the scan-backward workspace probes (bf16 + fp32) checked in process
# 0 while process 1 keeps ONE other kernel mix running: which co-running
# kernels go with the rare carry differences?
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6racebg}
mkdir -p $O
cd $R
export BG=1 NPROC=2 ONLY0="${ONLY0:-workspace}" REPS0=${REPS0:-600}
i=0
IFS=";" read -ra MIX <<< "${MIXES:-scan fwd;gemm nt;attn;skinny,conv;dropout,embed,colsum,grouped;ln+film;scan bwd C2 (du;scan bwd C2 fp32}"
for mix in "${MIX[@]}"; do
  i=$((i + 1))
  echo "== mix $i: $mix" | tee -a $O/bg.txt
  ONLY1="$mix" timeout -k 10 330 python -u tools/dbg/race_probe.py > $O/bg$i.txt 2>&1 || { tail -20 $O/bg$i.txt; exit 1; }
  grep -E "runs differ|background" $O/bg$i.txt | tee -a $O/bg.txt
done
