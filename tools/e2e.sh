#!/bin/bash
# drop-in app checks + the end-to-end line with its breakdown
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-e2e}
mkdir -p $O
T=""; for t in ${TESTS:-tests/test_app_gpu.py}; do T="$T $R/$t"; done
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 $R/bench.py --mode e2e --no-cpu --steps 2 --warmup 1 > $O/bench_e2e.json 2> $O/bench_e2e.err || { echo E2E_FAILED; tail $O/bench_e2e.err; exit 1; }
cat $O/bench_e2e.json
