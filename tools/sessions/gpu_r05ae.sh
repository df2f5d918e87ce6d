#!/bin/bash
# Round 5: C3 on 4 streams -- fused level-0 blocks (bench --fuse-l0 0/1/2) and fp16 Winograd at
# level 4 on/off (--wino-f16-levels ''), interleaved x3 on one box (both measured on 2 streams only)
set -u
O=${O:-gpurun_out/r05ae}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b c; do
  run f2$r 200 $C3
  run f1$r 200 $C3 --fuse-l0 1
  run f0$r 200 $C3 --fuse-l0 0
  run f2nw$r 200 $C3 --wino-f16-levels ''
done
