set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "conv" tests/test_gpu_configs.py > gpurun_out/t1.log 2>&1
tail -2 gpurun_out/t1.log
for i in 1 2; do
timeout -k 10 120 python -u tools/bench_conv.py 2>&1 | grep conv | sed 's/^/new /'
MTTS_LIB=mamba-tts-project_amd/mtts/libmtts_old.so timeout -k 10 120 python -u tools/bench_conv.py 2>&1 | grep conv | sed 's/^/old /'
done
