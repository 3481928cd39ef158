#!/bin/bash
# Measurement set, part A (one gpurun call): all GPU tests, the default
# bench line (with CPU baselines), rocprofv3 kernel stats of the default line and
# FETCH_SIZE / WRITE_SIZE passes (separate --pmc runs, kernel trace only).
# PART=B instead: the text workload's stats + PMC passes and the secondary lines.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2r}
mkdir -p $O
prof() {  # $1 = data, $2 = extra bench args
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$1 -o run -- python3 $R/bench.py --data $1 --no-cpu --no-900k $2 > $O/stats_$1.log 2>&1 || { echo STATS_$1_FAILED; tail $O/stats_$1.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$1 -o run -- python3 $R/bench.py --data $1 --no-cpu --no-900k --no-verify --steps 1 --warmup 1 > $O/pmc_fetch_$1.log 2>&1 || { echo FETCH_$1_FAILED; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$1 -o run -- python3 $R/bench.py --data $1 --no-cpu --no-900k --no-verify --steps 1 --warmup 1 > $O/pmc_write_$1.log 2>&1 || { echo WRITE_$1_FAILED; exit 1; }
}
if [ "${PART:-A}" = R ]; then
  prof random ""
elif [ "${PART:-A}" = A ]; then
  timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
  prof random ""
  cat $O/bench.json
else
  prof text ""
  timeout -k 10 200 python3 $R/bench.py --data text --no-cpu > $O/bench_text.json 2> $O/bench_text.err || exit 1
  timeout -k 10 200 python3 $R/bench.py --data mixed --no-cpu > $O/bench_mixed.json 2> $O/bench_mixed.err || exit 1
  timeout -k 10 200 python3 $R/bench.py --mode decompress --no-cpu > $O/bench_dec.json 2> $O/bench_dec.err || exit 1
  timeout -k 10 200 python3 $R/bench.py --mode decompress --data text --no-cpu > $O/bench_dec_text.json 2> $O/bench_dec_text.err || exit 1
  timeout -k 10 300 python3 $R/bench.py --mode e2e --no-cpu --steps 2 --warmup 1 > $O/bench_e2e.json 2> $O/bench_e2e.err || exit 1
  timeout -k 10 300 python3 $R/bench.py --unit 100000 --no-cpu > $O/bench_900k.json 2> $O/bench_900k.err || exit 1
  cat $O/bench_*.json
fi
echo done
