#!/bin/bash
# Round 6 call q: same-box recheck of C3 (the final run read 484 vs 503-506 earlier) with the
# headline and C2 beside it.
set -u
O=gpurun_out/r06q; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
run c3_1 200 python bench.py $C3
run hl 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt
run c3_2 200 python bench.py $C3
run c2 200 python bench.py --height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt
run c3_3 200 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-pairs 1 --no-alt
exit 0
