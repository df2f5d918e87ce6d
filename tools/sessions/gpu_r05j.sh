#!/bin/bash
# Round 5: bisect the fp16 range-flag failure of kind 10 with one workgroup per CU in the C3 forward
set -u
O=${O:-gpurun_out/r05j}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1) $(grep -o 'RuntimeError.*' $O/$name.log | head -1 | cut -c1-80)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
export RRIN_LIB_AB=ab/librrin_hip_hbpc1.so
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 5 --warmup 2 --no-alt --cpu-baseline off --wino-f16-kind 10"
run s1_l34 200 $C3 --wino-f16-levels 3,4 --streams 1
run s2_l4 200 $C3 --wino-f16-levels 4
run s2_l3 200 $C3 --wino-f16-levels 3
run s1_l3 200 $C3 --wino-f16-levels 3 --streams 1
run s2_l34_b2 200 $C3 --wino-f16-levels 3,4 --batch 2 --streams 1
run s1_l34_b1 200 $C3 --wino-f16-levels 3,4 --batch 1 --streams 1
