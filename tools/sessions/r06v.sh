#!/bin/bash
# Round 6 call v: the fused level-0 block with zero-C first MFMAs (conv a's chunk 0 peeled, conv
# b's first tap) vs the previous build: block0 tests, C3, C5.
set -u
O=gpurun_out/r06v; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run tb0 300 python -u -m pytest tests/test_gpu_block0.py -m gpu -x -q --timeout 120 --timeout-method thread
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run c3_new$k 200 python bench.py $C3
run c3_prev$k 200 env RRIN_LIB_AB=ab/librrin_hip_prev.so python bench.py $C3
done
run c5_new 300 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt
run c5_prev 300 env RRIN_LIB_AB=ab/librrin_hip_prev.so python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt
exit 0
