#!/bin/bash
# A/B of library variants (VARS: "prod" = libbz2mi.so, else libbz2mi_ab_<v>.so):
# a parity check against cpu_ref (PARITY=1), bench lines (DATAS) and, with
# TRAFFIC=1, FETCH_SIZE / WRITE_SIZE passes per stage (tools/traffic.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6ab}
mkdir -p $O
for v in ${VARS:-prod}; do
  lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi_ab_$v.so
  [ "$v" = prod ] && lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so
  export BZ2MI_LIBRARY=$lib
  if [ -n "$PARITY" ]; then
    (cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread ${PARITY_TESTS:-tests/test_gpu.py::test_seeded_inputs_match_cpuref tests/test_pins.py} -m gpu > $O/parity_$v.log 2>&1) || { echo PARITY_FAILED $v; tail -30 $O/parity_$v.log; exit 1; }
    echo "$v parity: $(tail -1 $O/parity_$v.log)"
  fi
  for d in ${DATAS:-realtext}; do
    timeout -k 10 200 python3 $R/bench.py --data $d --steps ${STEPS:-3} --warmup 1 --no-cpu --no-900k --no-units --no-verify ${ABARGS} > $O/b_${v}_$d.json 2> $O/b_${v}_$d.err || { echo BENCH_FAILED $v $d; tail -5 $O/b_${v}_$d.err; exit 1; }
    echo "$v $d: $(python3 -c "import json; d=json.load(open('$O/b_${v}_$d.json')); print(d['value'], d['roofline']['stage_ms'])")"
    if [ -n "$TRAFFIC" ]; then
      name=${v}_$d
      for k in FETCH_SIZE:fetch WRITE_SIZE:write; do
        c=${k%%:*}; kk=${k##*:}
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${kk}_$name -o run -- python3 $R/bench.py --data $d $ABARGS --no-cpu --no-900k --no-units --no-verify --steps 1 --warmup 1 > $O/pmc_${kk}_$name.log 2>&1 || { echo ${c}_FAILED $name; exit 1; }
        f=$(find $O/pmc_${kk}_$name -name "*counter_collection.csv" | head -1); mkdir -p $O/pmc_${kk}_x_$name; cp $f $O/pmc_${kk}_x_$name/run_counter_collection.csv; rm -rf $O/pmc_${kk}_$name
      done
      (cd $R && python3 tools/traffic.py $O $O/traffic_$name.json _x_$name $name "--data $d $ABARGS" > /dev/null) || { echo TRAFFIC_FAILED $name; exit 1; }
      echo "traffic $name: $(python3 -c "import json; d=json.load(open('$O/traffic_$name.json')); print({k: (round(v['fetch_bytes']/1e9,2), round(v['write_bytes']/1e9,2)) for k, v in d['stages'].items()})")"
    fi
  done
done
