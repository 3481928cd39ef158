# Build libbz2mi.so variants of one source file with extra -D flags, for A/B
# runs on the GPU box (BZ2MI_LIBRARY=build_v/<name>/libbz2mi.so).
#   tools/variants.sh bwt name1 "-DFOO" name2 "-DBAR -DBAZ" ...
set -e
cd "$(dirname "$0")/../bzip2-opencl_amd"
make -s -j8 >/dev/null
src=$1; shift
OBJS=$(ls build/*.o | grep -v "build/$src.o")
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p ../build_v/$name
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../include $flags \
    -c csrc/$src.hip -o ../build_v/$name/$src.o &
done
wait
for d in ../build_v/*/; do
  [ -f $d/$src.o ] && /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/libbz2mi.so $OBJS $d/$src.o
done
ls ../build_v
