#!/bin/bash
# Round 6 call al: persistent kind-14 workgroups for short K (next tile's raw(0), raw(1), U(0) in
# flight under the epilogue; two-phase exchange).  Kind-14 tests (persistent bitwise), headline A/B
# auto vs one-workgroup-per-tile (policy 3) interleaved, grid 256 / 1024 libraries, C2, per conv.
set -u
O=gpurun_out/r06al; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -4 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
run t42 400 python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q --timeout 120 --timeout-method thread
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_auto$k 200 python bench.py $HL
run hl_p3_$k 200 python bench.py $HL --wino42-geom 3
done
run hl_wg256 200 env RRIN_LIB_AB=ab/librrin_hip_wg256.so RRIN_LIB_AB_ABI=19 python bench.py $HL
run hl_wg1024 200 env RRIN_LIB_AB=ab/librrin_hip_wg1024.so RRIN_LIB_AB_ABI=19 python bench.py $HL
run hl_auto3 200 python bench.py $HL
C2="--height 368 --width 640 --batch 1 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
run c2_auto 200 python bench.py $C2
run c2_p3 200 python bench.py $C2 --wino42-geom 3
SH="32:32:0:1:25,64:32:0:1:25,32:32:0:2:25,64:64:1:1:25,128:64:1:1:25,64:64:1:3:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_nopers.so --batch 2 --rounds 5 --shapes $SH
exit 0
