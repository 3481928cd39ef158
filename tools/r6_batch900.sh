#!/bin/bash
# 900 KB mode on realtext: BWT time against the batch size (BZ2MI_BATCH_BLOCKS),
# i.e. how much of the gathered text stays in the caches
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6b900}
mkdir -p $O
for bb in ${BBS:-0 600 300 150}; do
  if [ "$bb" = 0 ]; then unset BZ2MI_BATCH_BLOCKS; else export BZ2MI_BATCH_BLOCKS=$bb; fi
  timeout -k 10 300 python3 $R/bench.py --data ${DATA:-realtext} --unit 100000 --no-cpu --no-units --no-900k --steps 3 --warmup 1 > $O/b_$bb.json 2> $O/b_$bb.err || { echo FAILED $bb; tail $O/b_$bb.err; exit 1; }
  echo "$bb: $(python3 -c "import json; d=json.load(open('$O/b_$bb.json')); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms'])")"
done
