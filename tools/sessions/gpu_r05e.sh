#!/bin/bash
# Round 5: one stream with the persistent exact-fp32 tile (kind 12) vs two streams of kind 6;
# C5 share (3840x2176 x 1) fp16 with / without the level-3/4 Winograd convs.
set -u
O=${O:-gpurun_out/r05e}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run s1_p 200 $B --streams 1
run s2_k6 200 $B --no-wino-persistent
run s1_k6 200 $B --streams 1 --no-wino-persistent
run s1_p_b 200 $B --streams 1
run s2_k6_b 200 $B --no-wino-persistent
run s4_p 200 $B --streams 4
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt"
run c5_w 300 $C5
run c5_d 300 $C5 --no-wino
run c5_w2 300 $C5
run c5_d2 300 $C5 --no-wino
