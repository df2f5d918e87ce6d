#!/bin/bash
# Round 5: headline (exact fp32, 1280x720 x 4) on 3 streams (parts 2 + 1 + 1 / 1 + 1 + 2) vs 2; C3 on 3 vs 4
set -u
O=${O:-gpurun_out/r05x}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run hl_s2$r 200 $B
  run hl_s3$r 200 $B --streams 3
  run hl_p112$r 200 $B --split 1,1,2
  run c3_s4$r 200 $C3
  run c3_s3$r 200 $C3 --streams 3
done
