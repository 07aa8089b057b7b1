#!/bin/bash
# Timing-only variants of libmtts.so (one source rebuilt with diag macros):
#   tools/diag_build.sh NAME "-DFLAG ..." [source.hip, default scan.hip]
#     ->  mamba-tts-project_amd/mtts/libmtts_NAME.so
# Use with MTTS_LIB=<path> (mtts/_lib.py), e.g. from tools/scan_lib_ab.py or
# tools/bench_mgemm.py.  Outputs of these builds are wrong by design.  Macros:
#   scan.hip: MTTS_DIAG_{NOMEM,NOCOMPUTE,NOSCALAR,NODPP,NOEXP}, MTTS_C1_DIAG_{NODMA,NOSTORE},
#             MTTS_FWD_NB=<tile buffers>
#   gemm.hip: MTTS_GEMM_DIAG_{NODMA,NOREAD,NOBAR,FIXK,SAMETILE}
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/mamba-tts-project_amd/mtts/csrc
SRC=${3:-scan.hip}
OBJ=${SRC%.hip}.o
make -C $CS -j8 >/dev/null
mkdir -p $CS/build/diag_$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$CS -w $2 -c $CS/$SRC -o $CS/build/diag_$1/$OBJ
objs=$(ls $CS/build/*.o | grep -v "/$OBJ\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/mamba-tts-project_amd/mtts/libmtts_$1.so $objs $CS/build/diag_$1/$OBJ
echo built libmtts_$1.so
