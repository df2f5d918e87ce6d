#!/bin/bash
# Round 4 session o: kind 8 with the register pressure cut (offsets recomputed per use,
# 32-bit store offsets): Winograd sweeps, per-conv A/B vs kind 3, whole forward.
set -u
O=${O:-gpurun_out/r04o}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -8 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread -k "conv or tail"
S=64:32:0:1,32:32:0:1,32:32:0:2,16:32:0:1
run ab_720 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,25 --batch 2 --shapes $S --rounds 7 --reps 5
run ab_c2 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,25 --batch 1 --height 368 --width 640 --shapes $S --rounds 9 --reps 10
exit 0
