#!/bin/bash
# A/B of environment settings on the default bench line: VARIANTS="name:ENV=v,ENV2=w name2:..."
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python3 $R/bench.py --no-cpu --no-900k ${ARGS} > $O/$name.json 2> $O/$name.err || { echo FAILED $name; tail -3 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['decode_check'], d['roofline']['stage_ms'])"
done
