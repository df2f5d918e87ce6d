#!/bin/bash
# s_setprio A/B on the 8-wave Winograd tile: p1 around each MFMA cluster, p2 static for waves 4-7
set -u
O=gpurun_out/r03w; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
S=32:32:0:1:20,64:32:0:1:20,16:32:0:1:20,64:128:0:4:20,64:64:1:2:20,128:64:1:1:20,128:128:2:2:20,256:128:2:1:20,256:256:3:1:20,512:256:3:1:20,512:512:4:1:20
run ab 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_p1.so,ab/librrin_hip_p2.so --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5
A='import sys, rrin_amd._lib as L; L.LIB_PATH = sys.argv[1]; sys.argv = ["bench.py"] + sys.argv[2:]; import bench; bench.main()'
ARGS="--cpu-baseline off --no-alt"
run c1_a 200 python bench.py $ARGS
run c1_p1 200 python -c "$A" ab/librrin_hip_p1.so $ARGS
run c1_p2 200 python -c "$A" ab/librrin_hip_p2.so $ARGS
run c1_a2 200 python bench.py $ARGS
run c1_p12 200 python -c "$A" ab/librrin_hip_p1.so $ARGS
run c1_p22 200 python -c "$A" ab/librrin_hip_p2.so $ARGS
