#!/bin/bash
# quick GPU check: the compressor's parity tests (TESTS= overrides), then the
# random and text bench lines
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick}
mkdir -p $O
T=${TESTS:-"$R/tests/test_gpu.py $R/tests/test_pins.py"}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for d in random text; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu --no-900k --data $d > $O/bench_$d.json 2> $O/bench_$d.err || { echo BENCH_FAILED $d; tail $O/bench_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$d.json')); print('$d', d['value'], d['ms_per_step'], d['config']['decode_check'], d['roofline']['stage_ms'])"
done
