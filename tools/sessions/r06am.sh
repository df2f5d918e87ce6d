#!/bin/bash
# Round 6 call am: how far the persistent short-K kind 14 should reach -- convs of up to 16 / 32
# chunks at the headline part (A/B libraries), and C2's level 0 (920 tiles) with the tile floor
# at 768.  Interleaved on one box.
set -u
O=gpurun_out/r06am; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -4 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
AB="RRIN_LIB_AB_ABI=19"
for k in 1 2; do
run hl_ch8_$k 200 python bench.py $HL
run hl_ch16_$k 200 env RRIN_LIB_AB=ab/librrin_hip_ch16.so $AB python bench.py $HL
run hl_ch32_$k 200 env RRIN_LIB_AB=ab/librrin_hip_ch32.so $AB python bench.py $HL
done
C2="--height 368 --width 640 --batch 1 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run c2_1024_$k 200 python bench.py $C2
run c2_768_$k 200 env RRIN_LIB_AB=ab/librrin_hip_mint768.so $AB python bench.py $C2
done
exit 0
