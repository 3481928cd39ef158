#!/bin/bash
# kernel stats of bench.py runs: KS="name:lib:args;..." (lib: prod or a variant name)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5ks}; mkdir -p $O
IFS=";" read -ra RS <<< "$KS"
for spec in "${RS[@]}"; do
  name=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=${rest#*:}
  L=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so; [ "$lib" = prod ] || L=$R/bzip2-opencl_amd/bz2mi/libbz2mi_$lib.so
  rm -rf $O/prof_$name
  BZ2MI_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 $R/bench.py --no-cpu --no-900k --no-units --steps 3 --warmup 1 $args > $O/ks_$name.json 2> $O/ks_$name.err || { echo KS_FAILED $name; tail -5 $O/ks_$name.err; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_stats.csv" | head -1)
  cp $f $O/ks_$name.csv
  rm -rf $O/prof_$name
  python3 - $O/ks_$name.csv $name <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2])
for r in rows[:14]:
    print(f"  {r['Name'].split('(')[0].replace('bz2mi::', '')[:36]:36s} calls {r['Calls']:>5} avg {float(r['AverageNs'])/1e6:8.3f} ms total {int(r['TotalDurationNs'])/1e6:8.2f}")
PY
done
