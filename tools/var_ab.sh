# A/B of library variants (VARS) on text and realtext BWT (1 GiB, 3 steps)
cd $GRAFT_REPO_ROOT
for v in ${VARS:-base}; do
  for d in ${DATAS:-text realtext}; do
    BZ2MI_LIBRARY=$PWD/bzip2-opencl_amd/bz2mi/libbz2mi_$v.so timeout -k 10 150 python3 bench.py --data $d --steps 3 --warmup 1 --no-cpu --no-900k --no-units --no-verify > gpurun_out/ab_$v_$d.json 2>/dev/null || { echo FAIL $v $d; exit 1; }
    echo "$v $d: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_$v_$d.json')); print(d['value'], d['roofline']['stage_ms']['bwt'])")"
  done
done
