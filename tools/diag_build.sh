#!/bin/bash
# Timing-only variants of libmtts.so (scan.hip rebuilt with a diag macro):
#   tools/diag_build.sh NAME "-DFLAG ..."  ->  mamba-tts-project_amd/mtts/libmtts_NAME.so
# Use with MTTS_LIB=<path> (mtts/_lib.py).  Outputs of these builds are wrong by design.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/mamba-tts-project_amd/mtts/csrc
make -C $CS -j8 >/dev/null
mkdir -p $CS/build/diag_$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$CS -w $2 -c $CS/scan.hip -o $CS/build/diag_$1/scan.o
objs=$(ls $CS/build/*.o | grep -v '/scan.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/mamba-tts-project_amd/mtts/libmtts_$1.so $objs $CS/build/diag_$1/scan.o
echo built libmtts_$1.so
