#!/bin/bash
# Round 6 call g: the ring from scratch inside the sub-pixel conv's launch (ABI 17 ring_full; the
# Net's fp16 / split16 sub-pixel up convs): kernel tests, the GPU suite, C3 A/B vs the r06d build.
set -u
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_ring timeout -k 10 300 python -u -m pytest tests/test_gpu_h8.py -m gpu -x -q --timeout 120 --timeout-method thread -k "subpixel"
step pytest_gpu timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bitwise_stream timeout -k 10 240 python tools/stream_bitwise.py --precision fp16 --height 736 --width 1280 --batch 4 --rounds 4
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
step c3_new1 timeout -k 10 200 python bench.py $C3
step c3_r06d1 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
step c3_new2 timeout -k 10 200 python bench.py $C3
step c3_r06d2 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
step c3_new3 timeout -k 10 200 python bench.py $C3
step c3_r06d3 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
step c5_new timeout -k 10 300 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt
step c5_r06d env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 300 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt
exit 0
