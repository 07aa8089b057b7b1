set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_modules.py > gpurun_out/t2.log 2>&1
tail -2 gpurun_out/t2.log
DEC_STEPS=200 timeout -k 10 300 python -u tools/decode_ab.py split 2>&1 | grep -v amdgpu.ids
