set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "scan" tests/test_gpu_configs.py > gpurun_out/t1.log 2>&1
tail -2 gpurun_out/t1.log
for i in 1 2; do
timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep bwd | sed 's/^/bcast /'
MTTS_LIB=mamba-tts-project_amd/mtts/libmtts_ldsred.so timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep bwd | sed 's/^/both /'
MTTS_LIB=mamba-tts-project_amd/mtts/libmtts_old.so timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep bwd | sed 's/^/old /'
done
