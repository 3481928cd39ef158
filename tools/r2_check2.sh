#!/bin/bash
# GPU tests (all), bench (default line with cpu + reference-on-GPU baselines),
# e2e through app.cpp, 900 KB mode line, rocprof stats of the default line.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --mode e2e --no-cpu --steps 2 --warmup 1 > $O/bench_e2e.json 2> $O/bench_e2e.err || { echo E2E_FAILED; tail $O/bench_e2e.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --unit 100000 --no-cpu > $O/bench_900k.json 2> $O/bench_900k.err || { echo B900_FAILED; tail $O/bench_900k.err; exit 1; }
cat $O/bench.json $O/bench_e2e.json $O/bench_900k.json
