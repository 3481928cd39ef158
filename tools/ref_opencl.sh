#!/bin/bash
# The reference itself, unmodified (app.cpp + kernel.cpp built from
# /root/reference by oracle/Makefile into oracle/_ref/ref_app), compressing on
# the MI355X through the ROCm OpenCL runtime; outputs compared with the O_ref
# fixtures / pins.  Small inputs first; stop at the first failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/refcl
rm -rf $O; mkdir -p $O/w
G=tests/golden
run() {  # name src level p
  cp $2 $O/w/$1
  timeout -k 10 ${TMO:-120} oracle/_ref/ref_app $O/w/$1 -k -s $3 -p $4 > $O/$1.s$3.p$4.log 2>&1
  rc=$?
  echo "$1 -s $3 -p $4 rc=$rc"
  [ $rc -eq 0 ] || return 1
  mv $O/w/$1.bz2 $O/w/$1.s$3.p$4.bz2
  sha256sum $O/w/$1.s$3.p$4.bz2 | cut -c1-64 > $O/w/$1.s$3.p$4.sha
}
run c1_text10k.bin $G/inputs/c1_text10k.bin 1 10 || exit 1
cmp $O/w/c1_text10k.bin.s1.p10.bz2 $G/oref/c1_text10k.s1.p10.bz2 && echo "C1 IDENTICAL to O_ref" || echo "c1_text10k.bin -s 1 -p 10 DIFFERS"
run text64k.bin $G/inputs/text64k.bin 9 10 || exit 1
cmp $O/w/text64k.bin.s9.p10.bz2 $G/oref/text64k.s9.p10.bz2 && echo "text64k s9 p10 IDENTICAL" || echo "text64k.bin -s 9 -p 10 DIFFERS"
run text64k.bin $G/inputs/text64k.bin 1 1 || exit 1
cmp $O/w/text64k.bin.s1.p1.bz2 $G/oref/text64k.s1.p1.bz2 && echo "text64k s1 p1 IDENTICAL" || echo "text64k.bin -s 1 -p 1 DIFFERS"
run text64k.bin $G/inputs/text64k.bin 1 10 || exit 1
cmp $O/w/text64k.bin.s1.p10.bz2 $G/oref/text64k.s1.p10.bz2 && echo "text64k s1 p10 IDENTICAL" || echo "text64k.bin -s 1 -p 10 DIFFERS"
run acgt64k.bin $G/inputs/acgt64k.bin 1 10 || exit 1
cmp $O/w/acgt64k.bin.s1.p10.bz2 $G/oref/acgt64k.s1.p10.bz2 && echo "acgt64k s1 p10 IDENTICAL" || echo "acgt64k.bin -s 1 -p 10 DIFFERS"
run rnd64k.bin $G/inputs/rnd64k.bin 1 10 || exit 1
cmp $O/w/rnd64k.bin.s1.p10.bz2 $G/oref/rnd64k.s1.p10.bz2 && echo "rnd64k s1 p10 IDENTICAL" || echo "rnd64k.bin -s 1 -p 10 DIFFERS"
ls -la $O/w
exit 0
