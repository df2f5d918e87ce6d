#!/bin/bash
# TH-4 Winograd tile (cfg 21): parity of every Winograd cfg, A/B of cfg 20 vs 21
# on the Net's conv shapes at 640x368 x 1 (C2) levels 1-4, C2 bench with / without.
set -u
O=gpurun_out/r03k; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run h8 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
S=32:64:1:1,64:64:1:2,128:64:1:1,128:256:1:4,64:128:2:1,128:128:2:2,256:128:2:1,256:512:2:4,128:256:3:1,256:256:3:1,256:256:3:2,512:256:3:1,512:1024:3:4,256:512:4:1,512:512:4:1
run ab_c2 300 python tools/conv_lab.py cfgab --cfgs 20,21 --precision fp32 --height 368 --width 640 --batch 1 --shapes $S --rounds 7 --check
run ab_c1 300 python tools/conv_lab.py cfgab --cfgs 20,21 --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5 --check
run c2_th4 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off
run c2_no 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-wino-th4
run c2_th4b 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off
exit 0
