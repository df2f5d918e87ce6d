#!/bin/bash
# Round 5: scheduler strategy A/B, second pass (the product now builds conv_winoc.hip with
# max-ilp): headline vs conv_wino.hip (kinds 3/4) max-memory-clause; C3 vs conv_f16.hip (record
# conv) max-ilp / max-memory-clause, conv_block0.hip max-ilp, conv_winoh.hip max-ilp; x3, one box
set -u
O=${O:-gpurun_out/r05ai}; mkdir -p $O; export TMPDIR=/tmp
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
  run hl_base$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_mc3.so run hl_mc3$r 200 $B
  run c3_base$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_f16ilp.so run c3_f16ilp$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_f16mc.so run c3_f16mc$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_b0ilp.so run c3_b0ilp$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_whilp.so run c3_whilp$r 200 $C3
done
