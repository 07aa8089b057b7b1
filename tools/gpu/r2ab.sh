set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/c2prof
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- python3 $GRAFT_REPO_ROOT/tools/gemm_step_ab.py hip 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
