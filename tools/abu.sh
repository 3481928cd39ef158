#!/bin/bash
# unit-protocol line at N=1: MTF waves per block and units per GPU
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abu; mkdir -p $O
for v in "u4:4:0" "u4g1:4:1" "u4g2:4:2" "u2:2:0" "u8:8:0"; do
  IFS=: read name k g <<< "$v"
  if [ "$g" != 0 ]; then export BZ2MI_MTF_WAVES=$g; else unset BZ2MI_MTF_WAVES; fi
  timeout -k 10 300 python3 $R/bench.py --no-cpu --no-900k --units-per-gpu $k > $O/$name.json 2> $O/$name.err || { echo FAIL $name; tail -3 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['decode_check'], d['roofline']['stage_ms_rank0'])"
done
