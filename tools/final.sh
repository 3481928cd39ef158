#!/bin/bash
# round-end check: every GPU test, smoke(), the default bench line
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest $R/tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['config']['decode_check'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['stage_ms'], d['cpu_baseline']['value'])"
