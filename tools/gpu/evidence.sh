#!/bin/bash
# Round-2 evidence pass: full -m gpu suite, the default bench line, rocprofv3
# kernel stats of that same bench command, and the FETCH_SIZE / WRITE_SIZE
# passes + kernel trace of the roofline kernel (north-star scan fwd).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/evidence
mkdir -p $O/pmc
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 $PT tests -m gpu > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bprof -o bench -- python3 $R/bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
for dt in bf16 fp32; do
  ITERS=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/f_$dt -o fetch_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/f_$dt.log 2>&1 || { tail -5 $O/pmc/f_$dt.log; exit 1; }
  ITERS=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/w_$dt -o write_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/w_$dt.log 2>&1 || { tail -5 $O/pmc/w_$dt.log; exit 1; }
  ITERS=20 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc/t_$dt -o trace_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/t_$dt.log 2>&1 || { tail -5 $O/pmc/t_$dt.log; exit 1; }
done
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete; du -sh $O; find $O -name "*.csv" -size +1M
