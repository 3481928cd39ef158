#!/bin/bash
# kernel timelines (rocprofv3 --kernel-trace, csv) of the N = 1 unit protocol
# and of the single call on the same data: UT="name:args;..." (bench.py args)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5ut}; mkdir -p $O
IFS=";" read -ra RS <<< "$UT"
for spec in "${RS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  rm -rf $O/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$name -o run -- python3 $R/bench.py --no-cpu --no-900k --no-units --no-verify --steps 3 --warmup 1 $args > $O/ut_$name.json 2> $O/ut_$name.err || { echo UT_FAILED $name; tail -5 $O/ut_$name.err; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_trace.csv" | head -1)
  python3 - $f $O/ut_$name.tsv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
with open(sys.argv[2], "w") as o:
    for r in rows:
        o.write(f"{r['Kernel_Name'].split('(')[0].replace('bz2mi::', '')}\t{r['Start_Timestamp']}\t{r['End_Timestamp']}\t{r.get('Queue_Id', '')}\t{r.get('Stream_Id', '')}\n")
PY
  rm -rf $O/prof_$name
  cat $O/ut_$name.json | head -c 400; echo
done
