#!/bin/bash
# Round 5 check H: segmented RLE1 emission -- seeded inputs (runs, long runs,
# zeros, mixed), 900 KB mode, app pins, C4 8 GiB through the unit protocol,
# then the mixed/random front-end A/B against the round-start front end.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu.py tests/test_app_gpu.py tests/test_fullsize_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "${TESTK:-seeded or 900k_mode_matches or periodic or pins or c4 or small_batches}" > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="prod oldfe" DATAS="mixed random" tools/var_ab.sh || exit 1
