#!/bin/bash
# Round 6 call ac: with the 2-stream fp16 default, re-check the fp16 schedule knobs at C3 --
# Winograd levels (4 / 3,4) and the fused level-0 blocks (FUSE_L0 2 / 1 / 0).
set -u
O=gpurun_out/r06ac; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run def_$k 200 python bench.py $C3
run w34_$k 200 python bench.py $C3 --wino-f16-levels 3,4
run f1_$k 200 python bench.py $C3 --fuse-l0 1
run f0_$k 200 python bench.py $C3 --fuse-l0 0
done
exit 0
