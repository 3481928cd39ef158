# Like tools/variants.sh, for flags that several source files must share:
#   tools/variants2.sh "decode dapi" name1 "-DFOO" name2 "-DBAR" ...
set -e
cd "$(dirname "$0")/../bzip2-opencl_amd"
make -s -j8 >/dev/null
srcs=$1; shift
OBJS=$(ls build/*.o)
for f in $srcs; do OBJS=$(echo "$OBJS" | grep -v "build/$f.o"); done
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p ../build_v/$name
  for f in $srcs; do
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../include $flags \
      -c csrc/$f.hip -o ../build_v/$name/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../build_v/$name/libbz2mi.so $OBJS $(for f in $srcs; do echo ../build_v/$name/$f.o; done)
done
ls ../build_v
