#!/bin/bash
# Round 5 check D: text-kernel phase sums (realtext, text) on the phase build
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d; mkdir -p $O
for d in ${DATAS:-realtext text}; do
  BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_ph.so DATA=$d MIB=${MIB:-256} timeout -k 10 150 python3 tools/tbkstat.py > $O/tbkstat_$d.txt 2>&1 || { echo TBKSTAT_FAIL $d; tail $O/tbkstat_$d.txt; exit 1; }
  echo "== $d"; grep -v amdgpu.ids $O/tbkstat_$d.txt
done
