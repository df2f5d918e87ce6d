#!/bin/bash
# Round 6 call t: kind 14 with AGPR accumulators (RRIN_WINO42_AGPR=1: 120 VGPRs + 96 AGPRs, no
# accumulator moves in the loop since the zero-C first MFMA) vs the VGPR product build.
set -u
O=gpurun_out/r06t; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run t42 300 env RRIN_LIB_AB=ab/librrin_hip_agpr.so python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q --timeout 120 --timeout-method thread
SH="32:32:0:1:25,64:32:0:1:25,64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:128:2:1:25,256:256:3:1:25,512:256:3:1:25,512:512:4:1:25,256:512:2:4:25,64:64:1:2:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_agpr.so --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_vgpr$k 200 python bench.py $HL
run hl_agpr$k 200 env RRIN_LIB_AB=ab/librrin_hip_agpr.so python bench.py $HL
done
run c2_vgpr 200 python bench.py $C2
run c2_agpr 200 env RRIN_LIB_AB=ab/librrin_hip_agpr.so python bench.py $C2
exit 0
