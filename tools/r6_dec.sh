#!/bin/bash
# decoder A/B: decode tests on the product library (TESTS=1), then the
# decompress lines (DATAS) for each library variant (VARS: prod or ab_<v>)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6dec}
mkdir -p $O
if [ -n "$TESTS" ]; then
  (cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_decode_gpu.py tests/test_app_gpu.py -m gpu > $O/tests.log 2>&1) || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
  echo "tests: $(tail -1 $O/tests.log)"
fi
for v in ${VARS:-prod}; do
  lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi_ab_$v.so
  [ "$v" = prod ] && lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so
  for d in ${DATAS:-realtext random}; do
    BZ2MI_LIBRARY=$lib timeout -k 10 300 python3 $R/bench.py --mode decompress --no-cpu --data $d --steps ${STEPS:-3} --warmup 1 > $O/dec_${v}_$d.json 2> $O/dec_${v}_$d.err || { echo DEC_FAILED $v $d; tail $O/dec_${v}_$d.err; exit 1; }
    echo "$v $d: $(python3 -c "import json; d=json.loads(open('$O/dec_${v}_$d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config'].get('round_trip_equal'), d.get('stage_ms'))")"
  done
done
