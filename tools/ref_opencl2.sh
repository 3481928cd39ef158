#!/bin/bash
# The unmodified reference (oracle/_ref/ref_app: app.cpp + kernel.cpp built
# from /root/reference) compressing on the MI355X through the ROCm OpenCL
# runtime.  (1) streams for the parity fixtures tests/golden/refgpu/ (block
# split, CRCs, BWT/origPtr, MTF symbols checked against O_ref by
# tests/test_refgpu.py); (2) the reference's own GPU throughput at its thesis
# setting p = 1024.  Stops at the first failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/refcl2
rm -rf $O; mkdir -p $O/w
python3 - <<'PY' || exit 1
import sys
sys.path.insert(0, "tests/golden"); sys.path.insert(0, "bzip2-opencl_amd")
import make_pins
from bz2mi import synth
O = "gpurun_out/refcl2/w/"
open(O + "txt2m75.bin", "wb").write(make_pins.make_input("txt2m75"))
open(O + "mix2m75.bin", "wb").write(make_pins.make_input("mix2m75"))
open(O + "rnd1m.bin", "wb").write(synth.random_bytes(1 << 20, 0x5EED2001).tobytes())
open(O + "rnd64m.bin", "wb").write(synth.random_bytes(64 << 20, 0x5EED2002).tobytes())
open(O + "txt64m.bin", "wb").write(synth.text_bytes(64 << 20, 0x5EED2003).tobytes())
PY
for f in c1_text10k text64k acgt64k rnd64k runs64k all_bytes; do cp tests/golden/inputs/$f.bin $O/w/; done
run() {  # file level p
  local t0=$(date +%s%N)
  timeout -k 10 ${TMO:-300} oracle/_ref/ref_app $O/w/$1 -k -s $2 -p $3 > $O/$1.s$2.p$3.log 2>&1
  local rc=$?
  local t1=$(date +%s%N)
  echo "$1 -s $2 -p $3 rc=$rc ms=$(( (t1 - t0) / 1000000 )) bytes=$(stat -c %s $O/w/$1)" | tee -a $O/times.txt
  [ $rc -eq 0 ] || return 1
  mv $O/w/$1.bz2 $O/w/$1.s$2.p$3.bz2
}
for f in c1_text10k text64k acgt64k rnd64k runs64k all_bytes; do
  run $f.bin 1 10 || exit 1
  run $f.bin 9 1 || exit 1
done
run txt2m75.bin 9 1 || exit 1
run mix2m75.bin 9 1 || exit 1
run rnd1m.bin 9 1 || exit 1
run rnd1m.bin 9 10 || exit 1
TMO=600 run rnd64m.bin 9 1024 || exit 1
TMO=600 run txt64m.bin 9 1024 || exit 1
# the 64 MiB runs: check they decode (libbz2) and keep only their hashes (gpurun_out merges <= 64 MiB)
python3 - <<'PY'
import bz2, hashlib
O = "gpurun_out/refcl2/w/"
with open(O + "../big.txt", "w") as f:
    for n in ("rnd64m", "txt64m"):
        z = open(O + n + ".bin.s9.p1024.bz2", "rb").read()
        ok = bz2.decompress(z) == open(O + n + ".bin", "rb").read()
        f.write(f"{n} -s 9 -p 1024 bytes={len(z)} sha256={hashlib.sha256(z).hexdigest()} decodes={ok}\n")
PY
rm -f $O/w/rnd64m.bin $O/w/txt64m.bin $O/w/rnd64m.bin.s9.p1024.bz2 $O/w/txt64m.bin.s9.p1024.bz2
cat $O/big.txt
ls -la $O/w
exit 0
