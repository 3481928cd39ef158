# rocprofv3 kernel statistics of the compress bench, random and text
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in ${DATAS:-random text}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$d -o run -- python3 $R/bench.py --data $d --steps 3 --warmup 1 --no-cpu --no-verify > $R/gpurun_out/prof_$d.log 2>&1 || exit 1
done
