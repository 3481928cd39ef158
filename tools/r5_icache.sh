#!/bin/bash
# counters available on the box, then an instruction-cache pass of the random
# bench (kernel trace only), to tools/issue-like csv under gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5ic}; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $O/avail.txt | sort -u > $O/ic_names.txt || true
cat $O/ic_names.txt
C=${IC_COUNTERS:-SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES}
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/pmc_ic -o run -- python3 $R/bench.py --data random --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_ic.log 2>&1 || { echo IC_FAILED; tail -5 $O/pmc_ic.log; exit 1; }
f=$(find $O/pmc_ic -name "*counter_collection.csv" | head -1)
python3 - $f <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.Counter())
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'].split('(')[0].replace('bz2mi::', '')[:30]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0))[:8]:
    print(k, dict(c))
PY
