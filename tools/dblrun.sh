# grid doubling checks: parity tests, per-round counts, kernel stats, tie-round A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_pins.py -m gpu > gpurun_out/t2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
BZ2MI_DBL_STATS=1 timeout -k 10 200 python3 bench.py --data realtext --unit 100000 --mib 256 --steps 1 --warmup 0 --no-cpu --no-900k --no-units > gpurun_out/dbl.json 2> gpurun_out/dbl.err || { echo DBL_FAILED; tail gpurun_out/dbl.err; exit 1; }
grep -v amdgpu.ids gpurun_out/dbl.err | head -20
TAG=ks9d RUNS="${KS:-rt900:--data realtext --unit 100000 --mib 256;t900:--data text --unit 100000 --mib 256}" bash tools/ks.sh || exit 1
for v in ${VARS:-tr1 tr3 tr6}; do
  for d in realtext text; do
    BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_$v.so timeout -k 10 200 python3 bench.py --data $d --unit 100000 --mib 256 --steps 3 --warmup 1 --no-cpu --no-900k --no-units --no-verify > gpurun_out/v_$v_$d.json 2>/dev/null || { echo VAR_FAILED $v $d; exit 1; }
    echo "$v $d: $(python3 -c "import json; d=json.load(open('gpurun_out/v_$v_$d.json')); print(d['value'], d['roofline']['stage_ms']['bwt'])")"
  done
done
