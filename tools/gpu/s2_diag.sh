#!/bin/bash
# scan fwd time decomposition (timing-only builds) + SQ counters of the real kernel
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M=$R/mamba-tts-project_amd/mtts
timeout -k 5 60 rocprofv3 -L > gpurun_out/s2/counters.txt 2>&1 || true
for v in base nomem nocomp; do
  lib=$M/libmtts.so; [ $v != base ] && lib=$M/libmtts_$v.so
  for dt in bf16 fp32; do
    MTTS_LIB=$lib timeout -k 10 120 python tools/scan_once.py $dt 2>&1 | grep scan | sed "s/^/$v /" || exit 1
  done
done
cd /tmp
ITERS=3 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/s2 -o pmcA -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/s2/pmcA.log 2>&1; echo "pmcA rc=$?"
ITERS=3 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/s2 -o pmcB -- python3 $R/tools/scan_once.py bf16 > $R/gpurun_out/s2/pmcB.log 2>&1; echo "pmcB rc=$?"
ls -R $R/gpurun_out/s2 | head -30
