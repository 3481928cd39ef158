#!/bin/bash
# Round 5: the unmodified reference (oracle/_ref/ref_app: app.cpp + kernel.cpp
# built from /root/reference) compressing wide-alphabet text and deep repeats
# on the MI355X through the ROCm OpenCL runtime -- streams for
# tests/golden/refgpu/ that pin the text BWT kernel (sparse pair index,
# deferred groups, resolve) to the reference's own bytes.  Stops at the first
# failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/refcl3
rm -rf $O; mkdir -p $O/w
python3 - <<'PY' || exit 1
import sys
sys.path.insert(0, "tests/golden"); sys.path.insert(0, "bzip2-opencl_amd")
import make_pins
from bz2mi import synth
O = "gpurun_out/refcl3/w/"
open(O + "rtx2m75.bin", "wb").write(make_pins.make_input("rtx2m75"))
open(O + "rep2m75.bin", "wb").write(make_pins.make_input("rep2m75"))
open(O + "rep64k.bin", "wb").write(synth.repeats_bytes(1 << 16).tobytes())
open(O + "rep1m.bin", "wb").write(synth.repeats_bytes(1 << 20).tobytes())
open(O + "rtx1m.bin", "wb").write(synth.realtext_bytes(1 << 20, 0x5EED3001).tobytes())
PY
cp tests/golden/inputs/rtext64k.bin $O/w/
run() {  # file level p
  local t0=$(date +%s%N)
  timeout -k 10 ${TMO:-300} oracle/_ref/ref_app $O/w/$1 -k -s $2 -p $3 > $O/$1.s$2.p$3.log 2>&1
  local rc=$?
  local t1=$(date +%s%N)
  echo "$1 -s $2 -p $3 rc=$rc ms=$(( (t1 - t0) / 1000000 )) bytes=$(stat -c %s $O/w/$1)" | tee -a $O/times.txt
  [ $rc -eq 0 ] || return 1
  mv $O/w/$1.bz2 $O/w/$1.s$2.p$3.bz2
}
run rtext64k.bin 9 1 || exit 1
run rtext64k.bin 1 10 || exit 1
run rep64k.bin 9 1 || exit 1
run rep64k.bin 1 10 || exit 1
run rep1m.bin 9 1 || exit 1
run rtx1m.bin 9 1 || exit 1
run rtx2m75.bin 9 1 || exit 1
run rep2m75.bin 9 1 || exit 1
python3 - <<'PY'
import bz2, glob, os
for z in sorted(glob.glob("gpurun_out/refcl3/w/*.bz2")):
    src = z.rsplit(".s", 1)[0]
    print(os.path.basename(z), len(open(z, "rb").read()), bz2.decompress(open(z, "rb").read()) == open(src, "rb").read())
PY
rm -f $O/w/*.bin
exit 0
