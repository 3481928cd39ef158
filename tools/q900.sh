# 900 KB mode checks: parity tests (incl. 1 GiB realtext at both units) and bench lines
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_pins.py tests/test_fullsize_gpu.py -m gpu -k "${TK:-not nothing}" > gpurun_out/t3.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
timeout -k 10 300 python3 bench.py --no-cpu --no-units --steps 5 --warmup 2 > gpurun_out/q_r.json 2> gpurun_out/q_r.err || { echo BENCH_FAILED; tail gpurun_out/q_r.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q_r.json')); print('random', d['value'], d['roofline']['stage_ms'], '900k', d['mode_900k']['value'], d['mode_900k']['stage_ms'])"
timeout -k 10 300 python3 bench.py --data realtext --no-cpu --no-units --steps 3 --warmup 1 > gpurun_out/q_rt.json 2> gpurun_out/q_rt.err || { echo BENCH_FAILED; tail gpurun_out/q_rt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q_rt.json')); print('realtext', d['value'], d['roofline']['stage_ms'], '900k', d['mode_900k']['value'], d['mode_900k']['stage_ms'])"
