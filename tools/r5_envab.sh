#!/bin/bash
# A/B of the single-call bench line under environment knobs:
# EAB="name:VAR=v VAR2=w;name2:..." on DATAS (default random), 3 steps, twice
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5eab}; mkdir -p $O
IFS=";" read -ra RS <<< "$EAB"
for rep in 1 2; do
for d in ${DATAS:-random}; do
for spec in "${RS[@]}"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python3 $R/bench.py --data $d --steps 3 --warmup 1 --no-cpu --no-900k --no-units --no-verify ${ARGS:-} > $O/eab_${name}_${d}_$rep.json 2> $O/eab_${name}_${d}_$rep.err || { echo EAB_FAILED $name; tail -5 $O/eab_${name}_${d}_$rep.err; exit 1; }
  echo "$name $d: $(python3 -c "import json; d=json.loads(open('$O/eab_${name}_${d}_$rep.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['stage_ms'])")"
done
done
done
