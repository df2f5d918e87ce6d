#!/bin/bash
# Round 5: same-box A/B of the Winograd source-view fix (current build) vs the build before it
# (ab/librrin_hip_old.so: net.hip + conv_f16.hip of ae5b651): headline and C3, interleaved
set -u
O=${O:-gpurun_out/r05ac}; mkdir -p $O; export TMPDIR=/tmp
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
for r in a b c; do
  run hl_new$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_old.so run hl_old$r 200 $B
  run c3_new$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_old.so run c3_old$r 200 $C3
done
