#!/bin/bash
# Round 5: level-4 split-K at 720p (576 kind-6 tiles on 512 slots), fp16 Winograd per conv at the
# C5 share and the C5 / C3 forward with Winograd at level 4 only.
set -u
O=${O:-gpurun_out/r05f}; mkdir -p $O; export TMPDIR=/tmp
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
run hl_s42 200 $B --wino-split 4:2
run hl_a2 200 $B
run hl_s42b 200 $B --wino-split 4:2
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt"
run c5_l4 300 $C5
run c5_d 300 $C5 --no-wino
run c5_l4b 300 $C5
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c3_l4 200 $C3
run c3_d 200 $C3 --no-wino
SH=128:256:3:1,256:256:3:1,256:256:3:3,512:256:3:0,256:512:4:1,512:512:4:1,256:512:2:4
timeout -k 10 300 python -u tools/conv_lab.py cfgab --precision fp16 --height 2176 --width 3840 --batch 1 --cfgs 10,11,4,23 --shapes $SH --rounds 5 --reps 3 > $O/cfgab_c5.log 2>&1; echo cfgab rc=$?
grep -v amdgpu $O/cfgab_c5.log | cut -c1-150
