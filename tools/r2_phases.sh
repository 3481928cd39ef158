#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/phases
mkdir -p $O
for d in random text; do
BZ2MI_LIBRARY=$R/build_v/phases/libbz2mi.so DATA=$d timeout -k 10 200 python3 $R/tools/phases.py > $O/$d.txt 2>&1 || { echo FAILED; tail $O/$d.txt; exit 1; }
echo "== $d"; cat $O/$d.txt
done
