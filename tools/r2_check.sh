#!/bin/bash
# Round 2 check set: GPU tests (incl. the stream-unit tests), smoke, the
# default bench line, a 2-rank rehearsal of the sharded single stream on one GPU.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_shard.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/shard_tests.log 2>&1 || { echo SHARD_TESTS_FAILED; tail -30 $O/shard_tests.log; exit 1; }
timeout -k 10 500 python -u -m pytest $R/tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
BZ2MI_SHARE_GPU=1 timeout -k 10 400 python3 $R/bench.py --gpus 2 --mib 512 --no-cpu > $O/bench_share2.json 2> $O/bench_share2.err || { echo SHARE_FAILED; tail -20 $O/bench_share2.err; exit 1; }
cat $O/bench.json $O/bench_share2.json
