#!/bin/bash
# Round 5: persistent tiles with ONE workgroup per CU (the other slot left to the other stream's
# kernels): exact fp32 kind 12 (ab/librrin_hip_bpc1.so) and fp16 kind 10 at levels 3-4
# (ab/librrin_hip_hbpc1.so) against the defaults, two streams, interleaved.
set -u
O=${O:-gpurun_out/r05h}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run hl_a 200 $B
RRIN_LIB_AB=ab/librrin_hip_bpc1.so run hl_p1 200 $B --wino-persistent 1
run hl_a2 200 $B
RRIN_LIB_AB=ab/librrin_hip_bpc1.so run hl_p1b 200 $B --wino-persistent 1
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c3_a 200 $C3
RRIN_LIB_AB=ab/librrin_hip_hbpc1.so run c3_p1 200 $C3 --wino-f16-kind 10 --wino-f16-levels 3,4
run c3_a2 200 $C3
RRIN_LIB_AB=ab/librrin_hip_hbpc1.so run c3_p1b 200 $C3 --wino-f16-kind 10 --wino-f16-levels 3,4
