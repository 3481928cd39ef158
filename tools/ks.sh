#!/bin/bash
# rocprofv3 kernel stats of short bench runs.  RUNS="name:bench args;..."
# writes gpurun_out/$TAG/<name>_kernel_stats.csv and prints the top kernels
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ks}
mkdir -p $O
IFS=';' read -ra RS <<< "${RUNS:-random:--data random}"
for spec in "${RS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  rm -rf $O/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 $R/bench.py --no-cpu --no-900k --no-units --steps 3 --warmup 1 $args > $O/$name.json 2> $O/$name.err || { echo FAIL $name; tail -5 $O/$name.err; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_stats.csv" | head -1)
  cp $f $O/${name}_kernel_stats.csv
  echo "== $name: $(python3 -c "import json; d=json.load(open('$O/$name.json')); print(d['value'], 'MB/s', d['ms_per_step'], 'ms', d['roofline']['stage_ms'])")"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(f"  {r['Name'].split('(')[0].replace('bz2mi::','')[:44]:44s} calls {int(r['Calls']):5d} avg_ms {float(r['AverageNs'])/1e6:8.3f} tot% {float(r['Percentage']):6.2f}")
PY
  rm -rf $O/prof_$name
done
