#!/bin/bash
# decompress benches of the tree under env settings (ENVS="A=1 B=2;C=3"), and build_v/dsym* libraries
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-decenv}
mkdir -p $O
IFS=';' read -ra SETS <<< "${ENVS:-}"
i=0
for e in "${SETS[@]}" ; do
  for d in ${DATASETS:-random text}; do
    env $e timeout -k 10 200 python3 $R/bench.py --mode decompress --data $d --no-cpu > $O/env${i}_$d.json 2> $O/env${i}_$d.err || { echo "BENCH $e $d FAILED"; tail -5 $O/env${i}_$d.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/env${i}_$d.json')); print('$e', '$d', d['value'], d.get('stage_ms'))"
  done
  i=$((i+1))
done
for v in $(ls $R/build_v 2>/dev/null | grep "${VPAT:-dsym}"); do
  for d in ${DATASETS:-random text}; do
    BZ2MI_LIBRARY=$R/build_v/$v/libbz2mi.so timeout -k 10 200 python3 $R/bench.py --mode decompress --data $d --no-cpu > $O/${v}_$d.json 2> $O/${v}_$d.err || { echo "BENCH $v $d FAILED"; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${v}_$d.json')); print('$v', '$d', d['value'], d.get('stage_ms'))"
  done
done
echo done
