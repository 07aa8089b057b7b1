set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tunable_ab.py gpurun_out/tunableop_results.csv 2>&1 | grep -v amdgpu.ids | tail -8
