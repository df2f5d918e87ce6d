#!/bin/bash
# Round 6 call ad: fp16 at 2 streams -- size-class tables (default / medium / xlarge), Winograd off at
# level 4; C5 with FUSE_L0 1 vs 2.
set -u
O=gpurun_out/r06ad; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
C5="--height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt"
for k in 1 2; do
run def_$k 200 python bench.py $C3
run med_$k 200 python bench.py $C3 --size-class medium
run xl_$k 200 python bench.py $C3 --size-class xlarge
run now_$k 200 python bench.py $C3 --wino-f16-levels ""
done
run c5_f1 300 python bench.py $C5
run c5_f2 300 python bench.py $C5 --fuse-l0 2
exit 0
