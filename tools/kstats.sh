#!/bin/bash
# rocprofv3 kernel stats of short bench runs (DATA list), summaries printed
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in ${DATA:-random text}; do
  rm -rf $R/gpurun_out/ks_$d
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$d -o run -- python3 $R/bench.py --no-cpu --no-900k --data $d --steps 3 --warmup 1 $EXTRA > $R/gpurun_out/ks_$d.log 2>&1 || { echo FAIL $d; tail -5 $R/gpurun_out/ks_$d.log; exit 1; }
  f=$(find $R/gpurun_out/ks_$d -name "*kernel_stats.csv" | head -1)
  echo "== $d"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f\"{r['Name'][:60]:60s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1000:9.1f}\")
"
done
