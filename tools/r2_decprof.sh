#!/bin/bash
# rocprofv3 kernel stats of the decompress bench (DATA)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-decprof}
mkdir -p $O
for d in ${DATASETS:-random}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$d -o run -- python3 $R/bench.py --mode decompress --data $d --no-cpu --steps 3 --warmup 1 > $O/stats_$d.log 2>&1 || { echo STATS_FAILED; tail $O/stats_$d.log; exit 1; }
done
echo done
