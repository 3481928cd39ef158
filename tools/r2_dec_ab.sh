#!/bin/bash
# decoder GPU tests, then decompress benches of the tree and build_v/dsym*
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-decab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in tree $(ls $R/build_v 2>/dev/null | grep dsym); do
  lib=$R/build_v/$v/libbz2mi.so
  [ $v = tree ] && lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so
  for d in ${DATASETS:-random text}; do
    BZ2MI_LIBRARY=$lib timeout -k 10 200 python3 $R/bench.py --mode decompress --data $d --no-cpu > $O/${v}_$d.json 2> $O/${v}_$d.err || { echo "BENCH $v $d FAILED"; tail -5 $O/${v}_$d.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${v}_$d.json')); print('$v', '$d', d['value'], d['roofline'].get('stage_ms'))"
  done
done
echo done
