# Kernel statistics for the C3 (text) and C4 (mixed) workloads.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in ${DATASETS:-text}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$d -o run -- python3 $R/bench.py --data $d --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/prof_$d.log 2>&1 || exit 1
done
