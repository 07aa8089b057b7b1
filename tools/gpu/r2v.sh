set -e -o pipefail
cd $GRAFT_REPO_ROOT
L=mamba-tts-project_amd/mtts
for v in noxw noxwls noxwlp noxwlsp; do
  echo "== ${v:-product}"
  if [ -z "$v" ]; then timeout -k 10 120 python -u tools/gemv_ab.py; else MTTS_LIB=$L/libmtts_$v.so timeout -k 10 120 python -u tools/gemv_ab.py; fi
done 2>&1 | grep -v amdgpu.ids
