# BWT parity tests, then compress benches (random, text) and the text kernel
# statistics.  BZ2MI_WLEVEL=0 selects the workgroup level kernel for A/B runs.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for d in random text; do
  for w in ${WLEVELS:-1}; do
    BZ2MI_WLEVEL=$w timeout -k 10 200 python3 $R/bench.py --data $d --no-cpu > $O/b_${d}_$w.json 2> $O/b_${d}_$w.err || exit 1
  done
done
DATASETS=text bash $R/tools/prof_text.sh
