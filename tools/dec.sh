#!/bin/bash
# decoder checks: decoder + app tests, then the decompress lines (random, text)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-dec}
mkdir -p $O
T=""; for t in ${TESTS:-tests/test_decode_gpu.py tests/test_app_gpu.py}; do T="$T $R/$t"; done
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for d in random text; do
  timeout -k 10 300 python3 $R/bench.py --mode decompress --no-cpu --data $d > $O/dec_$d.json 2> $O/dec_$d.err || { echo DEC_FAILED $d; tail $O/dec_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/dec_$d.json')); print('$d', d['value'], d['ms_per_step'], d['config']['round_trip_equal'], d['stage_ms'])"
done
