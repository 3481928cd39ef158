#!/bin/bash
# quick check: compressor GPU tests + random / text / mixed bench lines
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu.py $R/tests/test_shard.py $R/tests/test_pins.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for d in random text mixed; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu --data $d > $O/bench_$d.json 2> $O/bench_$d.err || { echo BENCH_${d}_FAILED; tail $O/bench_$d.err; exit 1; }
done
python3 -c "
import json
for d in ['random', 'text', 'mixed']:
    x = json.load(open('$O/bench_' + d + '.json')); print(d, x['value'], x['ms_per_step'], x['roofline']['stage_ms'])
"
