set -e -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "gemm_rows or packed" 2>&1 | tail -1
bash tools/gpu/scan_c2_fwd.sh
