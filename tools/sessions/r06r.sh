#!/bin/bash
# Round 6 call r: kind 14 without the 96 accumulator-zeroing moves per tile (chunk 0's first MFMA
# of each point takes C = 0) vs the previous build (ab/librrin_hip_prev.so): kind-14 tests,
# per-conv abconv (bitwise), whole forward; plus the same-box C3 recheck.
set -u
O=gpurun_out/r06r; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run t42 300 python -u -m pytest tests/test_gpu_wino42.py tests/test_gpu_h8.py -m gpu -x -q --timeout 120 --timeout-method thread
SH="32:32:0:1:25,64:32:0:1:25,64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:256:3:1:25,512:512:4:1:25,256:512:2:4:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_prev.so --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_new$k 200 python bench.py $HL
run hl_prev$k 200 env RRIN_LIB_AB=ab/librrin_hip_prev.so python bench.py $HL
run c3_$k 200 python bench.py $C3
done
exit 0
