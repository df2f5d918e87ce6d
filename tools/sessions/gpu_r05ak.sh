#!/bin/bash
# Round 5: C3 on 4 streams with GPU_MAX_HW_QUEUES 4 / 8 (bench default) / 16 (bench --hw-queues), x3
set -u
O=${O:-gpurun_out/r05ak}; mkdir -p $O; export TMPDIR=/tmp
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
  run q8$r 200 $C3
  run q4$r 200 $C3 --hw-queues 4
  run q16$r 200 $C3 --hw-queues 16
done
