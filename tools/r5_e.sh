#!/bin/bash
# Round 5 check E: seeded/realtext parity of the product build, then phase
# sums and the A/B line of the phase build
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_fullsize_gpu.py tests/test_refgpu_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "${TESTK:-seeded or 900k_mode_matches or (realtext and 10000)}" > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="${VARS:-ph}" DATAS="realtext text" tools/var_ab.sh || exit 1
tools/r5_d.sh
