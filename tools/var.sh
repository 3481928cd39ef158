#!/bin/bash
# A/B of BWT variants (make variant VAR=...): text-kernel phase sums per
# variant library and workload.  VARS="ph pc64 ..." DATAS="realtext:64 ..."
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-var}
mkdir -p $O
for v in ${VARS:-ph}; do
  for dm in ${DATAS:-realtext:64 repeats:16}; do
    d=${dm%%:*}; m=${dm##*:}
    echo "== $v $d $m" | tee -a $O/var.log
    DATA=$d MIB=$m BZ2MI_LIBRARY=$R/bzip2-opencl_amd/bz2mi/libbz2mi_$v.so timeout -k 10 200 python3 $R/tools/tbkstat.py 2>&1 | grep -v amdgpu.ids | tee -a $O/var.log || exit 1
  done
done
