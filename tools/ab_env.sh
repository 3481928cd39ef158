# GPU tests, then compress benches (random, text) for each value of the env
# variable $VAR in $VALS (A/B of a launcher switch).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for d in ${DATAS:-random text}; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python3 $R/bench.py --data $d --no-cpu > $O/b_${d}_$v.json 2> $O/b_${d}_$v.err || exit 1
  done
done
