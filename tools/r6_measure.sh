#!/bin/bash
# Round-6 measurement set (one gpurun call): bench lines (C2 with the 900 KB
# mode and the N = 1 unit line + CPU baselines; C3 realtext; 27-symbol text;
# decompression of realtext (C5's workload) and random),
# rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes and the SQ/GRBM issue
# pass (separate --pmc runs, kernel trace only), turned into
# gpurun_out/$TAG/r06_{traffic,issue}_<name>.json on the box (stamped with the
# library's sha256, which bench.py checks) -- copy them to profiles/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6m}
mkdir -p $O
STEPS="--steps ${STEPS:-5} --warmup 2"
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python3 $R/bench.py $STEPS > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
echo "random: $(python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'], 'u', d['unit_protocol_n1']['value'] if d['unit_protocol_n1'] else None, '900k', d['mode_900k']['value'])")"
timeout -k 10 400 python3 $R/bench.py --data realtext --no-cpu --no-units $STEPS > $O/bench_realtext.json 2> $O/bench_realtext.err || { echo BENCH_RT_FAILED; tail $O/bench_realtext.err; exit 1; }
echo "realtext: $(python3 -c "import json; d=json.load(open('$O/bench_realtext.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'], '900k', d['mode_900k']['value'], d['mode_900k']['roofline']['stage_ms'])")"
timeout -k 10 300 python3 $R/bench.py --data text --no-cpu --no-units --no-900k $STEPS > $O/bench_text.json 2> $O/bench_text.err || { echo BENCH_TXT_FAILED; tail $O/bench_text.err; exit 1; }
echo "text: $(python3 -c "import json; d=json.load(open('$O/bench_text.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'])")"
for d in realtext random; do
timeout -k 10 300 python3 $R/bench.py --mode decompress --data $d --no-cpu $STEPS > $O/bench_dec_$d.json 2> $O/bench_dec_$d.err || { echo BENCH_DEC_FAILED; tail $O/bench_dec_$d.err; exit 1; }
echo "decompress $d: $(python3 -c "import json; d=json.loads(open('$O/bench_dec_$d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('stage_ms'))")"
done
fi
IFS=";" read -ra RS <<< "${RUNS:-random:--data random;realtext:--data realtext;text:--data text;random900k:--data random --unit 100000;realtext900k:--data realtext --unit 100000}"
for spec in "${RS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  rm -rf $O/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 $R/bench.py --no-cpu --no-900k --no-units --steps 3 --warmup 1 $args > $O/ks_$name.json 2> $O/ks_$name.err || { echo KS_FAILED $name; tail -5 $O/ks_$name.err; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_stats.csv" | head -1)
  cp $f $O/r06_kernel_stats_$name.csv
  rm -rf $O/prof_$name
done
IFS=";" read -ra PS <<< "${PMC:-random:--data random;realtext:--data realtext;text:--data text;random900k:--data random --unit 100000;realtext900k:--data realtext --unit 100000}"
for spec in "${PS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$name -o run -- python3 $R/bench.py $args --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_fetch_$name.log 2>&1 || { echo FETCH_${name}_FAILED; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$name -o run -- python3 $R/bench.py $args --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_write_$name.log 2>&1 || { echo WRITE_${name}_FAILED; exit 1; }
  for k in fetch write; do f=$(find $O/pmc_${k}_$name -name "*counter_collection.csv" | head -1); mkdir -p $O/pmc_${k}_x_$name; cp $f $O/pmc_${k}_x_$name/run_counter_collection.csv; rm -rf $O/pmc_${k}_$name; done
  (cd $R && python3 tools/traffic.py $O $O/r06_traffic_$name.json _x_$name $name "$args" > /dev/null) || { echo TRAFFIC_${name}_FAILED; exit 1; }
  echo "traffic $name: $(python3 -c "import json; d=json.load(open('$O/r06_traffic_$name.json')); print({k: round(v['traffic_bytes']/1e9, 2) for k, v in d['stages'].items()})")"
done
IFS=";" read -ra IS <<< "${ISSUE:-random:--data random;realtext:--data realtext;random900k:--data random --unit 100000}"
for spec in "${IS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_issue_$name -o run -- python3 $R/bench.py $args --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_issue_$name.log 2>&1 || { echo ISSUE_${name}_FAILED; exit 1; }
  f=$(find $O/pmc_issue_$name -name "*counter_collection.csv" | head -1)
  cp $f $O/issue_$name.csv
  rm -rf $O/pmc_issue_$name
  (cd $R && python3 tools/issue.py $O/issue_$name.csv $O/r06_issue_$name.json "SQ/GRBM pass of bench.py $args (1 GiB, -9, p=10)" > /dev/null) || { echo ISSUEPY_${name}_FAILED; exit 1; }
  rm -f $O/issue_$name.csv
done
echo done
