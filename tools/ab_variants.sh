# Compress benches of the build_v/* library variants (tools/variants.sh) and
# the in-tree library ("tree"), DATASETS (default: random text).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abv
mkdir -p $O
for v in tree $(ls $R/build_v); do
  lib=$R/build_v/$v/libbz2mi.so
  [ $v = tree ] && lib=$R/bzip2-opencl_amd/bz2mi/libbz2mi.so
  for d in ${DATASETS:-random text}; do
    BZ2MI_LIBRARY=$lib timeout -k 10 200 python3 $R/bench.py --data $d --no-cpu $BENCH_ARGS > $O/${v}_$d.json 2> $O/${v}_$d.err || exit 1
  done
done
