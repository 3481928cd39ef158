#!/bin/bash
# stage times against input size (tail / occupancy model of each stage)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-sizes}
mkdir -p $O
for mib in ${SIZES:-256 512 590 768 1024}; do
  for data in ${DATAS:-random}; do
    timeout -k 10 300 python3 $R/bench.py --no-cpu --no-verify --data $data --mib $mib > $O/b_${data}_$mib.json 2> $O/b_${data}_$mib.err || { echo BENCH_FAILED $mib; tail $O/b_${data}_$mib.err; exit 1; }
    python3 -c "
import json
d = json.load(open('$O/b_${data}_$mib.json')); print('$data', $mib, d['config']['blocks'], d['value'], d['ms_per_step'], d['roofline']['stage_ms'])
"
  done
done
