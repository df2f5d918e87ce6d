#!/bin/bash
# Round 6 call h: in-launch ring fix-up with one K group per ring tile (config-independent bits):
# ring kernel tests, the GPU suite, fp16 stream bitwise, C3 / headline / C2 A/B vs the r06d build.
set -u
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_ring timeout -k 10 300 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_winoh.py -m gpu -x -q --timeout 120 --timeout-method thread -k "subpixel"
step pytest_gpu timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bitwise_stream timeout -k 10 240 python tools/stream_bitwise.py --precision fp16 --height 736 --width 1280 --batch 4 --rounds 4
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
for k in 1 2; do
step c3_new$k timeout -k 10 200 python bench.py $C3
step c3_r06d$k env RRIN_LIB_AB=ab/librrin_hip_r06d.so RRIN_LIB_AB_ABI=16 timeout -k 10 200 python bench.py $C3
step hl_new$k timeout -k 10 200 python bench.py $HL
step hl_r06d$k env RRIN_LIB_AB=ab/librrin_hip_r06d.so RRIN_LIB_AB_ABI=16 timeout -k 10 200 python bench.py $HL
step c2_new$k timeout -k 10 200 python bench.py $C2
step c2_r06d$k env RRIN_LIB_AB=ab/librrin_hip_r06d.so RRIN_LIB_AB_ABI=16 timeout -k 10 200 python bench.py $C2
done
exit 0
