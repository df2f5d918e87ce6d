#!/bin/bash
# Round 6 call x: same-box check of the final build vs the r06s build (before the zero-C MFMA
# changes outside kind 14) on the headline, C3 and C2.
set -u
O=gpurun_out/r06x; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_fin$k 200 python bench.py $HL
run hl_r06s$k 200 env RRIN_LIB_AB=ab/librrin_hip_r06s.so python bench.py $HL
run c3_fin$k 200 python bench.py $C3
run c3_r06s$k 200 env RRIN_LIB_AB=ab/librrin_hip_r06s.so python bench.py $C3
done
exit 0
