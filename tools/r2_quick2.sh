#!/bin/bash
# compressor + decoder GPU tests, compress benches (random, text), decompress benches (random, text)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu.py $R/tests/test_shard.py $R/tests/test_pins.py $R/tests/test_decode_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in compress decompress; do for d in random text; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu --mode $m --data $d > $O/${m}_$d.json 2> $O/${m}_$d.err || { echo BENCH_FAILED $m $d; tail $O/${m}_$d.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/${m}_$d.json')); print('$m', '$d', d['value'], d.get('roofline', {}).get('stage_ms') or d.get('stage_ms'))"
done; done
