#!/bin/bash
# A/B of the N = 1 unit protocol line under environment knobs:
# UAB="name:VAR=v VAR2=w;name2:..." (bench.py --units-per-gpu 4)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5uab}; mkdir -p $O
IFS=";" read -ra RS <<< "$UAB"
for rep in 1 2; do
for spec in "${RS[@]}"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 240 python3 $R/bench.py --units-per-gpu 4 --steps 5 --warmup 2 --no-cpu --no-900k --no-verify ${ARGS:-} > $O/uab_${name}_$rep.json 2> $O/uab_${name}_$rep.err || { echo UAB_FAILED $name; tail -5 $O/uab_${name}_$rep.err; exit 1; }
  python3 - $O/uab_${name}_$rep.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"].get("stage_ms_rank0"))
PY
done
done
