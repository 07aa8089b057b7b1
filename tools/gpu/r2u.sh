set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
DEC_STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/decprof -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_ab.py rowsonly > $GRAFT_REPO_ROOT/gpurun_out/decprof.log 2>&1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/decprof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | cut -c1-150 | head -16
