set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "gemm_rows or state_update or step" > gpurun_out/t1.log 2>&1
tail -3 gpurun_out/t1.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_modules.py > gpurun_out/t2.log 2>&1
tail -3 gpurun_out/t2.log
timeout -k 10 200 python -u tools/decode_ab.py shapes > gpurun_out/ab1.log 2>&1
cat gpurun_out/ab1.log
MTTS_GEMV_NT=1 timeout -k 10 200 python -u tools/decode_ab.py shapes > gpurun_out/ab2.log 2>&1
cat gpurun_out/ab2.log
DEC_STEPS=200 timeout -k 10 300 python -u tools/decode_ab.py packed > gpurun_out/ab3.log 2>&1
cat gpurun_out/ab3.log
