#!/bin/bash
# Round 5: forward stream count on the final build (headline fp32 and C3 fp16): 2 (default) vs 4
# (one pair per stream) vs 1; same box, interleaved.
set -u
O=${O:-gpurun_out/r05w}; mkdir -p $O; export TMPDIR=/tmp
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
  run hl_s2$r 200 $B --streams 2
  run hl_s4$r 200 $B --streams 4
  run c3_s2$r 200 $C3 --streams 2
  run c3_s4$r 200 $C3 --streams 4
done
run hl_s1 200 $B --streams 1
run c3_s1 200 $C3 --streams 1
