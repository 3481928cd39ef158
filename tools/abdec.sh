cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abdec; mkdir -p $O
for v in new; do
  if [ $v = base ]; then export BZ2MI_LIBRARY=$R/bzip2-opencl_amd/bz2mi/libbz2mi_base.so; else unset BZ2MI_LIBRARY; fi
  timeout -k 10 200 python3 $R/bench.py --mode decompress --no-cpu --data text > $O/$v.json 2> $O/$v.err || { echo FAIL $v; tail -3 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['value'], d['stage_ms'])"
done
