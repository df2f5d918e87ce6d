#!/bin/bash
# tile order A/B of the 8-wave Winograd tile: o1 column-fastest then co block, o2 co block outermost per image
set -u
O=gpurun_out/r03ab; mkdir -p $O; export TMPDIR=/tmp
S=32:32:0:1:20,64:32:0:1:20,64:64:1:2:20,128:64:1:1:20,128:128:2:2:20,256:128:2:1:20,256:512:2:4:20,256:256:3:1:20,512:256:3:1:20,512:512:4:1:20
timeout -k 10 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_o1.so,ab/librrin_hip_o2.so --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 7 > $O/ab.log 2>&1 || exit 1
A='import sys, rrin_amd._lib as L; L.LIB_PATH = sys.argv[1]; sys.argv = ["bench.py"] + sys.argv[2:]; import bench; bench.main()'
ARGS="--cpu-baseline off --no-alt"
for r in 1 2; do
  timeout -k 10 200 python bench.py $ARGS > $O/c1_a$r.log 2>&1 || exit 1
  timeout -k 10 200 python -c "$A" ab/librrin_hip_o1.so $ARGS > $O/c1_o1_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -c "$A" ab/librrin_hip_o2.so $ARGS > $O/c1_o2_$r.log 2>&1 || exit 1
done
grep -v amdgpu $O/ab.log
