set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "packed" > gpurun_out/t1.log 2>&1
tail -2 gpurun_out/t1.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_modules.py > gpurun_out/t2.log 2>&1
tail -2 gpurun_out/t2.log
DEC_STEPS=200 timeout -k 10 300 python -u tools/decode_ab.py xpacked > gpurun_out/ab3.log 2>&1
cat gpurun_out/ab3.log
cd /tmp && export TMPDIR=/tmp
DEC_STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/decprof3 -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_ab.py rowsonly > $GRAFT_REPO_ROOT/gpurun_out/decprof3.log 2>&1
