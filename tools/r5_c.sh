#!/bin/bash
# Round 5 check C: the text kernel's dynamic deal (libbz2mi_dyn: scalar item
# index) against cpu_ref at 6 MiB and 1 GiB of realtext, its speed and phase
# sums beside the static deal (libbz2mi_ph), then the experiment: the same loop
# with the item index as a VGPR broadcast (libbz2mi_dynv, trace build) under a
# watchdog.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c; mkdir -p $O
BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_dyn.so timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_fullsize_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "seeded or 900k_mode_matches or (realtext and 10000)" > $O/tests_dyn.log 2>&1 || { echo DYN_TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests_dyn.log | head -20; tail -20 $O/tests_dyn.log; exit 1; }
tail -1 $O/tests_dyn.log
BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_wqtr.so DATA=realtext MIB=64 HANG_S=20 REPS=1 timeout -k 10 120 python3 -u tools/tbktrace.py > $O/wqtr.log 2>&1 || { echo WQ_PROBE_FAILED; tail -30 $O/wqtr.log; exit 1; }
tail -2 $O/wqtr.log
BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_wq.so timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_fullsize_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "seeded or 900k_mode_matches or (realtext and 10000)" > $O/tests_wq.log 2>&1 || { echo WQ_TESTS_FAILED; grep -E "FAIL|Error|assert" $O/tests_wq.log | head -20; tail -20 $O/tests_wq.log; exit 1; }
tail -1 $O/tests_wq.log
VARS="ph dyn wq" DATAS="realtext text" tools/var_ab.sh || exit 1
for v in ph dyn wq; do
  BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_$v.so DATA=realtext MIB=256 timeout -k 10 120 python3 tools/tbkstat.py > $O/tbkstat_$v.txt 2>&1 || { echo TBKSTAT_FAIL $v; tail $O/tbkstat_$v.txt; exit 1; }
  echo "== $v"; cat $O/tbkstat_$v.txt
done
export BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_dynv.so
DATA=realtext MIB=1 HANG_S=20 REPS=1 timeout -k 10 90 python3 -u tools/tbktrace.py > $O/dynv.log 2>&1
echo "dynv rc=$?"; tail -30 $O/dynv.log
exit 0
