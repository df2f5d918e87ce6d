#!/bin/bash
# Winograd F(4x4,3x3) (cfg 22): conv parity of every config, error vs F(2x2),
# cfg 20 vs 22 timing on the Net's conv shapes at 1280x720 x 2 and 640x368 x 1
set -u
O=gpurun_out/r03n; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run h8 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
run err 120 python tools/w4_err.py
S=32:32:0:1,32:32:0:2,64:32:0:1,16:32:0:1,64:128:0:4,32:64:1:1,64:64:1:2,128:64:1:1,128:256:1:4,64:128:2:1,128:128:2:2,256:128:2:1,256:512:2:4,128:256:3:1,256:256:3:1,256:256:3:2,512:256:3:1,512:1024:3:4,256:512:4:1,512:512:4:1
run ab_c1 300 python tools/conv_lab.py cfgab --cfgs 20,22 --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5
run ab_c2 300 python tools/conv_lab.py cfgab --cfgs 20,22 --precision fp32 --height 368 --width 640 --batch 1 --shapes $S --rounds 5
exit 0
