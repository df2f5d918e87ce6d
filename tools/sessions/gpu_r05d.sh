#!/bin/bash
# Round 5: the full GPU suite with kind 12 (exact fp32 default) and fp16 Winograd at levels 3-4;
# whole-forward A/B of both, interleaved.
set -u
O=${O:-gpurun_out/r05d}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -3 | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run hl_a1 200 $B
run hl_b1 200 $B --no-wino-persistent
run hl_a2 200 $B
run hl_b2 200 $B --no-wino-persistent
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c3_a1 200 $C3
run c3_b1 200 $C3 --no-wino
run c3_c1 200 $C3 --wino-f16-kind 10
run c3_a2 200 $C3
run c3_b2 200 $C3 --no-wino
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c2_a 200 $C2
run c2_b 200 $C2 --no-wino-persistent
for f in $O/hl_*.log $O/c3_*.log $O/c2_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
