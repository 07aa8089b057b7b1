#!/bin/bash
# round-1 evidence (one-lane-per-channel scan forward): full GPU tests, bench line, rocprofv3 kernel stats of the
# same bench command, FETCH_SIZE / WRITE_SIZE passes of the roofline kernel
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s11
mkdir -p $O $O/pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o bench_prof -- python3 $R/bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo "profiled bench done"
for dt in bf16 fp32; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc -o trace_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/trace_$dt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o fetch_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/fetch_$dt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc -o write_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/write_$dt.log 2>&1 || exit 1
done
ls $O $O/pmc | head -40
