#!/bin/bash
# Round-6 evidence (one call): the full -m gpu suite + smoke, the default bench
# line, rocprofv3 kernel stats of that bench command, FETCH_SIZE / WRITE_SIZE +
# kernel trace of the roofline kernel (north-star scan fwd, fp32 and bf16),
# FETCH_SIZE / WRITE_SIZE / SQ passes + kernel trace of the C2 scan backward,
# SQ / MFMA PMC passes + kernel trace over C2 training steps, kernel traces of
# the C5 train.py step and of the C4 decode step.  Outputs: gpurun_out/${EVDIR:-ev6}/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${EVDIR:-ev6}
mkdir -p $O/pmc $O/c2 $O/c5 $O/dec $O/sbwd
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  grep smoke $O/smoke.log
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bprof -o bench -- python3 $R/bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
echo "bench profiled"
for dt in bf16 fp32; do
  ITERS=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o fetch_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/f_$dt.log 2>&1 || { tail -5 $O/pmc/f_$dt.log; exit 1; }
  ITERS=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc -o write_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/w_$dt.log 2>&1 || { tail -5 $O/pmc/w_$dt.log; exit 1; }
  ITERS=100 timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc -o trace_$dt -- python3 $R/tools/scan_once.py $dt > $O/pmc/t_$dt.log 2>&1 || { tail -5 $O/pmc/t_$dt.log; exit 1; }
done
echo "scan fwd pmc done"
ITERS=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/sbwd -o fetch -- python3 $R/tools/scan_bwd_once.py > $O/sbwd/f.log 2>&1 || { tail -5 $O/sbwd/f.log; exit 1; }
ITERS=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/sbwd -o write -- python3 $R/tools/scan_bwd_once.py > $O/sbwd/w.log 2>&1 || { tail -5 $O/sbwd/w.log; exit 1; }
ITERS=5 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sbwd -o sq -- python3 $R/tools/scan_bwd_once.py > $O/sbwd/sq.log 2>&1 || { tail -5 $O/sbwd/sq.log; exit 1; }
ITERS=50 timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sbwd -o trace -- python3 $R/tools/scan_bwd_once.py > $O/sbwd/t.log 2>&1 || { tail -5 $O/sbwd/t.log; exit 1; }
echo "scan bwd pmc done"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/c2 -o p1 -- python3 $R/tools/gemm_step_ab.py hip 1 > $O/c2/p1.log 2>&1 || { tail -5 $O/c2/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/c2 -o p2 -- python3 $R/tools/gemm_step_ab.py hip 1 > $O/c2/p2.log 2>&1 || { tail -5 $O/c2/p2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o kt -- python3 $R/tools/gemm_step_ab.py hip 20 > $O/c2/kt.log 2>&1 || { tail -5 $O/c2/kt.log; exit 1; }
echo "c2 done"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/c5_once.py > $O/c5/c5.log 2>&1 || { tail -5 $O/c5/c5.log; exit 1; }
DEC_STEPS=60 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 $R/tools/decode_ab.py rowsonly > $O/dec/dec.log 2>&1 || { tail -5 $O/dec/dec.log; exit 1; }
find $O -name "*kernel_trace.csv" -size +20M -delete; find $O -name "*.db" -delete; du -sh $O
