#!/bin/bash
# Round 6 call b: the cleaned product library (rejected kinds removed, ABI 16, conv_winoc under
# max-ilp) through the GPU suite, then the headline, C2 and C3 bench lines.
set -u
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench timeout -k 10 240 python bench.py --steps 20 --warmup 5
step bench_c2 timeout -k 10 240 python bench.py --height 368 --width 640 --batch 1 --steps 50 --warmup 10
step bench_c3 timeout -k 10 300 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5
exit 0
