#!/bin/bash
# compress GPU tests (quick set) + decoder A/B (r2_dec_ab.sh) + phases/compress A/B (r2_diag.sh)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-combo}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu.py $R/tests/test_pins.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=${TAG:-combo}_dec bash $R/tools/r2_dec_ab.sh || exit 1
TAG=${TAG:-combo}_diag DATASETS="${CDATA:-random}" bash $R/tools/r2_diag.sh
