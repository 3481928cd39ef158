#!/bin/bash
# quick check: GPU tests of the compressor + bench line + text line
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu.py $R/tests/test_shard.py $R/tests/test_pins.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 $R/bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --no-cpu --data text > $O/bench_text.json 2> $O/bench_text.err || { echo BENCHT_FAILED; tail $O/bench_text.err; exit 1; }
python3 -c "
import json
for f in ['$O/bench.json', '$O/bench_text.json']:
    d = json.load(open(f)); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'])
"
