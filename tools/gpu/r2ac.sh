set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py > gpurun_out/t1.log 2>&1
tail -2 gpurun_out/t1.log
timeout -k 10 300 python -u bench.py --skip-extras --steps 5 --warmup 2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-400
