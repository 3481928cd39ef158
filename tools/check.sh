#!/bin/bash
# GPU check (one gpurun call): all GPU tests, then the default bench line and
# the unit-protocol line at N = 1.  TESTS=... narrows the test selection.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-check}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-$R/tests} -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 $R/bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --no-cpu --no-900k --units-per-gpu 4 > $O/bench_units.json 2> $O/bench_units.err || { echo BENCHU_FAILED; tail $O/bench_units.err; exit 1; }
python3 -c "
import json
for f in ['$O/bench.json', '$O/bench_units.json']:
    d = json.load(open(f)); print(d['value'], d['ms_per_step'], d['config'].get('decode_check'), d['roofline'].get('stage_ms', d['roofline'].get('stage_ms_rank0')), (d.get('mode_900k') or {}).get('value'))
"
