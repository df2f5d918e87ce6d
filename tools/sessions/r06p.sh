#!/bin/bash
# Round 6 call p: kind-14 co-block group budget (RRIN_WINO42_UGROUP_KB: 0 = co blocks of a tile
# position consecutive, 512 / 2048 (default) / 8192 KB of U per group) in the whole forward; C2
# without the geometry split-K (kind 14 everywhere).
set -u
O=gpurun_out/r06p; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_def_$k 200 python bench.py $HL
for g in 0 512 8192; do
run hl_g${g}_$k 200 env RRIN_LIB_AB=ab/librrin_hip_w42g$g.so python bench.py $HL
done
done
run c2_def 200 python bench.py $C2
run c2_nosplit 200 python bench.py $C2 --wino-split none
run c2_def2 200 python bench.py $C2
run c2_nosplit2 200 python bench.py $C2 --wino-split none
exit 0
