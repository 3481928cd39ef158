#!/bin/bash
# kernel stats of the text bench line (rocprofv3 --kernel-trace --stats)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-textstats}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_${DATA:-text} -o run -- python3 $R/bench.py --data ${DATA:-text} --no-cpu --steps 3 --warmup 1 > $O/stats_${DATA:-text}.log 2>&1 || { echo STATS_FAILED; tail $O/stats_${DATA:-text}.log; exit 1; }
echo stats done
