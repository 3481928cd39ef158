#!/bin/bash
# Diagnostics: phase stamps (build_v/phases), A/B benches of the other
# build_v/* variants, SQ PMC passes of the in-tree build (256 MiB random).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-diag}
mkdir -p $O
if [ -f $R/build_v/phases/libbz2mi.so ]; then
  for d in random text; do
    BZ2MI_LIBRARY=$R/build_v/phases/libbz2mi.so DATA=$d timeout -k 10 200 python3 $R/tools/phases.py > $O/phases_$d.txt 2>&1 || { echo PHASES_FAILED; tail $O/phases_$d.txt; exit 1; }
    echo "== phases $d"; cat $O/phases_$d.txt
  done
fi
for v in tree $(ls $R/build_v 2>/dev/null | grep -v phases | grep "${VGREP:-.}"); do
  lib=$R/build_v/$v/libbz2mi.so
  [ $v = tree ] && lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so
  for d in ${DATASETS:-random text}; do
    [ "$d" = none ] && continue
    BZ2MI_LIBRARY=$lib timeout -k 10 200 python3 $R/bench.py --data $d --no-cpu --no-verify > $O/${v}_$d.json 2> $O/${v}_$d.err || { echo "BENCH $v $d FAILED"; tail -5 $O/${v}_$d.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${v}_$d.json')); print('$v', '$d', d['value'], d['roofline']['stage_ms'])"
  done
done
if [ -n "$PMC" ]; then
  run() {
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $O/$1 -o run -- \
      python3 $R/bench.py --steps 1 --warmup 0 --mib 256 --data ${PMCDATA:-random} --no-cpu --no-verify $PMCARGS > $O/$1.log 2>&1 || { echo "PASS $1 FAILED"; tail -5 $O/$1.log; exit 1; }
  }
  run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum"
  run p3 "SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
fi
echo done
