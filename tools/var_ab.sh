#!/bin/bash
# A/B of library variants (VARS; "prod" = the product libbz2mi.so) on DATAS
# (default text realtext), 1 GiB, 3 steps: compress MB/s and BWT ms
cd $GRAFT_REPO_ROOT
for v in ${VARS:-prod}; do
  lib=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_$v.so
  [ "$v" = prod ] && lib=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi.so
  for d in ${DATAS:-text realtext}; do
    BZ2MI_LIBRARY=$lib timeout -k 10 ${ABT:-150} python3 bench.py --data $d --steps 3 --warmup 1 --no-cpu --no-900k --no-units --no-verify ${ABARGS} > gpurun_out/ab_${v}_${d}.json 2>gpurun_out/ab_${v}_${d}.err || { echo FAIL $v $d; tail -5 gpurun_out/ab_${v}_${d}.err; exit 1; }
    echo "$v $d: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_${v}_${d}.json')); print(d['value'], d['roofline']['stage_ms'])")"
  done
done
