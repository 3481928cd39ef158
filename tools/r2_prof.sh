#!/bin/bash
# rocprofv3 kernel stats + FETCH/WRITE passes for a workload (DATA=random|text|mixed), tag TAG.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=${DATA:-text}
O=$R/gpurun_out/prof_${TAG:-r2}_$D
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --data $D --steps 2 --warmup 1 --no-cpu --no-verify > $O/stats.log 2>&1 || { echo STATS_FAILED; tail $O/stats.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --data $D --no-cpu --no-verify --steps 1 --warmup 1 > $O/pmc_fetch.log 2>&1 || { echo FETCH_FAILED; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --data $D --no-cpu --no-verify --steps 1 --warmup 1 > $O/pmc_write.log 2>&1 || { echo WRITE_FAILED; exit 1; }
grep -h '"metric"' $O/stats.log | head -2
echo done
