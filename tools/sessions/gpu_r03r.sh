#!/bin/bash
# ping-pong Winograd main loop (cfg 23, kind 6) vs cfg 20; Winograd split-K: parity, per-shape A/B, whole forward
set -u
O=gpurun_out/r03r; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
S=32:32:0:1,32:32:0:2,64:32:0:1,16:32:0:1,64:128:0:4,32:64:1:1,64:64:1:2,128:64:1:1,128:256:1:4,64:128:2:1,128:128:2:2,256:128:2:1,256:512:2:4,128:256:3:1,256:256:3:1,512:256:3:1,256:512:4:1,512:512:4:1
run split 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread
run ab 300 python tools/conv_lab.py cfgab --cfgs 20,23 --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5
run h8 400 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
run c1_k3 300 python bench.py --cpu-baseline off
run c1_k6 300 python bench.py --cpu-baseline off --wino-kind 6
run bd_c2 300 python tools/conv_lab.py breakdown --precision fp32 --height 368 --width 640 --batch 1
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off"
run c2_k3 300 python bench.py $C2
run c2_k6 300 python bench.py $C2 --wino-kind 6
run c2_s234 300 python bench.py $C2 --wino-split 2:2,3:4,4:8
run c2_s34 300 python bench.py $C2 --wino-split 3:4,4:8
run c2_s234b 300 python bench.py $C2 --wino-split 2:2,3:2,4:4
