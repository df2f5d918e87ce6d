#!/bin/bash
# Round 6, first call: the fenced product build (GPU suite, headline bench), then the max-ilp
# build of conv_winoc.hip (ab/librrin_hip_ilp_winoc.so, ISA-checked) through the GPU suite,
# tools/stream_bitwise.py and the headline (parity in the line), A/B interleaved with the product.
set -u
O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -2 $O/$n.log; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_prod1 timeout -k 10 240 python bench.py --steps 20 --warmup 5
export RRIN_LIB_AB=ab/librrin_hip_ilp_winoc.so
step bench_ilp1 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline off
step bitwise_ilp timeout -k 10 240 python tools/stream_bitwise.py --precision fp32 --height 720 --width 1280 --batch 4 --rounds 6
step pytest_gpu_ilp timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
unset RRIN_LIB_AB
step bench_prod2 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline off
export RRIN_LIB_AB=ab/librrin_hip_ilp_winoc.so
step bench_ilp2 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline off
unset RRIN_LIB_AB
step bench_prod3 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline off
exit 0
