set -e -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
for k in 4 2 1 8; do
MTTS_SCAN_BWD_SEGS=$k timeout -k 10 120 python -u tools/bench_scan.py quick 2>&1 | grep "bwd.*bfloat16" | sed "s/^/K=$k /"
done
done
