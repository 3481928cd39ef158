#!/bin/bash
# N = 1 unit line (4 units of 256 MiB on one MI355X) with host timelines
# (BZ2MI_UNIT_TRACE), under the stream-priority settings in PRIOS
# (BZ2MI_STREAM_PRIO digits: context stream, A, M, B, F; 0 default, 1 high, 2 low).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6ul}
mkdir -p $O
for pr in ${PRIOS:-01010 11010}; do
  BZ2MI_STREAM_PRIO=$pr BZ2MI_UNIT_TRACE=$O/tr_$pr timeout -k 10 300 python3 $R/bench.py --units-per-gpu ${UPG:-4} --steps 5 --warmup 2 --no-cpu > $O/bench_$pr.json 2> $O/bench_$pr.err || { echo FAILED $pr; tail -20 $O/bench_$pr.err; exit 1; }
  python3 $R/tools/unit_hops.py $O/tr_$pr > $O/hops_$pr.json || exit 1
  echo "$pr: $(python3 -c "import json; d=json.load(open('$O/bench_$pr.json')); print(d['value'], d['ms_per_step'])") $(cat $O/hops_$pr.json | tr -d '\n ')"
done
