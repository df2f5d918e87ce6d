#!/bin/bash
# fp16 tile-table sweep at the C3 per-stream part (1280x736 x 2) and the C3 bench before it
set -u
O=gpurun_out/r03x; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run c3 200 python bench.py --precision fp16 --height 736 --width 1280 --cpu-baseline off --no-alt
run tune 900 python tools/conv_lab.py tune --precision fp16 --height 736 --width 1280 --batch 2 --out $O/tune_fp16_1280x736x2.json
