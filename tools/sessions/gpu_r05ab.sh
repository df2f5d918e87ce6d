#!/bin/bash
# Round 5: fp16 medium-class tile table (sweep at 1280x736 x 1, the 4-stream C3 part) and fp16
# Winograd at levels 3-4 vs 4, interleaved C3 runs; C5 share (xxlarge class) with levels 3-4 vs 4
set -u
O=${O:-gpurun_out/r05ab}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 6 --warmup 2 --cpu-baseline off --no-alt"
for r in a b c; do
  run c3_large$r 200 $C3 --no-f16-medium-table
  run c3_med$r 200 $C3
  run c3_medw34$r 200 $C3 --wino-f16-levels 3,4
  run c3_largew34$r 200 $C3 --no-f16-medium-table --wino-f16-levels 3,4
done
for r in a b; do
  run c5_w4$r 200 $C5
  run c5_w34$r 200 $C5 --wino-f16-levels 3,4
done
