#!/bin/bash
# 3-stage Winograd ring with counted vmcnt waits + bare barrier (ab/librrin_hip_s3.so) vs the 2-stage product
set -u
O=gpurun_out/r03u; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
S=32:32:0:1:20,32:32:0:2:20,64:32:0:1:20,16:32:0:1:20,64:128:0:4:20,32:64:1:1:20,64:64:1:2:20,128:64:1:1:20,128:256:1:4:20,64:128:2:1:20,128:128:2:2:20,256:128:2:1:20,256:512:2:4:20,128:256:3:1:20,256:256:3:1:20,512:256:3:1:20,256:512:4:1:20,512:512:4:1:20
run ab 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_s3.so --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5
A='import sys, rrin_amd._lib as L; L.LIB_PATH = "ab/librrin_hip_s3.so"; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
ARGS="--cpu-baseline off --no-alt"
run c1_a 200 python bench.py $ARGS
run c1_b 200 python -c "$A" $ARGS
run c1_a2 200 python bench.py $ARGS
run c1_b2 200 python -c "$A" $ARGS
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c2_a 200 python bench.py $C2
run c2_b 200 python -c "$A" $C2
