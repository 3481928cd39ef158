#!/bin/bash
# compressor GPU tests, then bench lines for random / text / mixed
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-check3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu.py $R/tests/test_shard.py $R/tests/test_pins.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for data in ${DATAS:-random text mixed}; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu --data $data > $O/b_$data.json 2> $O/b_$data.err || { echo BENCH_FAILED $data; tail $O/b_$data.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$O/b_$data.json')); print('$data', d['value'], d['ms_per_step'], d['roofline']['stage_ms'])
"
done
