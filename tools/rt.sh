#!/bin/bash
# realtext round-4 check: BWT routing + parity at moderate size, then the
# GPU parity tests named in TESTS and the bench lines in DATA
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-rt}
mkdir -p $O
IFS=';' read -ra CK <<< "${CHECKS:-realtext 64;repeats 16}"
for c in "${CK[@]}"; do
  BZ2MI_BWT_STATS=1 timeout -k 10 300 python3 -u $R/tools/rt_check.py $c >> $O/check.log 2>&1 || { echo CHECK_FAILED $c; tail -20 $O/check.log; exit 1; }
done
cat $O/check.log
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -20 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for d in ${DATA:-}; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu --no-900k --data $d > $O/bench_$d.json 2> $O/bench_$d.err || { echo BENCH_FAILED $d; tail $O/bench_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$d.json')); print('$d', d['value'], d['ms_per_step'], d['config']['decode_check'], d['roofline']['stage_ms'])"
done
