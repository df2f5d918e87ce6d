#!/bin/bash
# Round 6 call af: kind 14 with the pixel-per-lane epilogue (coalesced 512-B store runs, 16 gather
# reads per lane) vs the previous build: kind-14 tests, per-conv abconv (bitwise), whole forward.
set -u
O=gpurun_out/r06af; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -12 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run t42 400 python -u -m pytest tests/test_gpu_wino42.py tests/test_gpu_h8.py -m gpu -x -q --timeout 120 --timeout-method thread
SH="32:32:0:1:25,64:32:0:1:25,32:32:0:2:25,64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:256:3:1:25,512:512:4:1:25,256:512:2:4:25,64:64:1:3:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_prev.so --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_new$k 200 python bench.py $HL
run hl_prev$k 200 env RRIN_LIB_AB=ab/librrin_hip_prev.so python bench.py $HL
done
exit 0
