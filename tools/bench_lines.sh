#!/bin/bash
# the bench lines (random, text, mixed, 900 KB mode), no CPU legs
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3base}
mkdir -p $O
for a in "--data random" "--data text" "--data mixed" "--unit 100000"; do
  f=$(echo $a | tr -d ' -')
  timeout -k 10 300 python3 $R/bench.py --no-cpu $a > $O/b_$f.json 2> $O/b_$f.err || { echo FAILED $a; tail $O/b_$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
done
