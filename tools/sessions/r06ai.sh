#!/bin/bash
# Round 6 call ai: kind 14 on 16 x 16 tiles where that needs fewer workgroup rounds (the level-4
# grids): kind-14 tests (geometries bitwise), headline A/B auto vs forced 32 x 8 (same box,
# interleaved), C2 A/B, then per-conv abconv auto vs the forced-32x8 library.
set -u
O=gpurun_out/r06ai; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -6 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run t42 400 python -u -m pytest tests/test_gpu_wino42.py tests/test_gpu_h8.py -m gpu -x -q --timeout 120 --timeout-method thread
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_auto$k 200 python bench.py $HL
run hl_wide$k 200 python bench.py $HL --wino42-geom 1
done
C2="--height 368 --width 640 --batch 1 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
run c2_auto 200 python bench.py $C2
run c2_wide 200 python bench.py $C2 --wino42-geom 1
SH="512:512:4:1:25,256:512:4:1:25,1024:512:4:1:25,256:256:3:1:25,128:128:2:1:25,64:64:1:1:25,32:32:0:1:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_wide.so --batch 2 --rounds 5 --shapes $SH
exit 0
