#!/bin/bash
# Round 5 check B: GPU tests of test_gpu.py (900 KB tiny blocks, memory
# pressure, seeded inputs incl. realtext/repeats), A/B of the text sort size,
# then the dynamic-deal trace probe.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b; mkdir -p $O
[ -n "$SKIPTESTS" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "${TESTK:-900k or golden or seeded}" > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
[ -n "$SKIPTESTS" ] || tail -1 $O/tests.log
VARS="${VARS:-prod ts512}" DATAS="${DATAS:-realtext text}" tools/var_ab.sh || exit 1
tools/r5_dyn.sh
