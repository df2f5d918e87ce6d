#!/bin/bash
# Round 6 call o: level-0 convs on kind 14 from cin 16 / 32 / 64 (default) in the whole forward.
set -u
O=gpurun_out/r06o; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
for k in 1 2; do
for m in 64 32 16; do
run hl_m${m}_$k 200 python bench.py $HL --wino42-min-cin-l0 $m
done
done
for m in 64 32 16; do
run c2_m${m} 200 python bench.py $C2 --wino42-min-cin-l0 $m
done
exit 0
