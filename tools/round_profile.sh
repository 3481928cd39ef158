# Round-end measurement set (one gpurun call): GPU tests, the default bench
# line, its rocprofv3 kernel stats, and FETCH_SIZE / WRITE_SIZE passes of the
# same command (separate --pmc runs, kernel trace only), plus the secondary
# workloads.  Everything lands in gpurun_out/round/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
timeout -k 10 500 python -u -m pytest $R/tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu > $O/stats.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --no-verify --steps 1 --warmup 1 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --no-verify --steps 1 --warmup 1 > $O/pmc_write.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/bench.py --data text --no-cpu > $O/bench_text.json 2>/dev/null
timeout -k 10 200 python3 $R/bench.py --data mixed --no-cpu > $O/bench_mixed.json 2>/dev/null
timeout -k 10 200 python3 $R/bench.py --mode decompress --no-cpu > $O/bench_dec.json 2>/dev/null
timeout -k 10 200 python3 $R/bench.py --mode decompress --data text --no-cpu > $O/bench_dec_text.json 2>/dev/null
exit 0
