#!/bin/bash
# Round-4 measurement set (one gpurun call): the default bench line (C2 with
# the 900 KB mode, the N = 1 unit-protocol line and the CPU baselines), the
# realtext (C3) and text lines, rocprofv3 kernel stats of random / realtext /
# random in the 900 KB mode, and FETCH_SIZE / WRITE_SIZE passes (separate
# --pmc runs, kernel trace only) of random and realtext.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r4m}
mkdir -p $O
STEPS="--steps ${STEPS:-5} --warmup 2"
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python3 $R/bench.py $STEPS > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
echo "random: $(python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'], 'u', d['unit_protocol_n1']['value'] if d['unit_protocol_n1'] else None, '900k', d['mode_900k']['value'])")"
timeout -k 10 400 python3 $R/bench.py --data realtext --no-cpu --no-units $STEPS > $O/bench_realtext.json 2> $O/bench_realtext.err || { echo BENCH_RT_FAILED; tail $O/bench_realtext.err; exit 1; }
echo "realtext: $(python3 -c "import json; d=json.load(open('$O/bench_realtext.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'], '900k', d['mode_900k']['value'], d['mode_900k']['stage_ms'])")"
timeout -k 10 300 python3 $R/bench.py --data text --no-cpu --no-units --no-900k $STEPS > $O/bench_text.json 2> $O/bench_text.err || { echo BENCH_TXT_FAILED; tail $O/bench_text.err; exit 1; }
echo "text: $(python3 -c "import json; d=json.load(open('$O/bench_text.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'])")"
fi
IFS=";" read -ra RS <<< "${RUNS:-random:--data random;realtext:--data realtext;text:--data text;random900k:--data random --unit 100000;realtext900k:--data realtext --unit 100000}"
for spec in "${RS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  rm -rf $O/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 $R/bench.py --no-cpu --no-900k --no-units --steps 3 --warmup 1 $args > $O/ks_$name.json 2> $O/ks_$name.err || { echo KS_FAILED $name; tail -5 $O/ks_$name.err; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_stats.csv" | head -1)
  cp $f $O/${name}_kernel_stats.csv
  rm -rf $O/prof_$name
done
for d in ${PMC:-random realtext}; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$d -o run -- python3 $R/bench.py --data $d --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_fetch_$d.log 2>&1 || { echo FETCH_$d_FAILED; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$d -o run -- python3 $R/bench.py --data $d --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_write_$d.log 2>&1 || { echo WRITE_$d_FAILED; exit 1; }
done
for d in ${ISSUE:-random realtext}; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_issue_$d -o run -- python3 $R/bench.py --data $d --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_issue_$d.log 2>&1 || { echo ISSUE_$d_FAILED; exit 1; }
  f=$(find $O/pmc_issue_$d -name "*counter_collection.csv" | head -1)
  cp $f $O/issue_$d.csv
  rm -rf $O/pmc_issue_$d
done
echo done
