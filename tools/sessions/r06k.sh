#!/bin/bash
# Round 6 call k: kind 14 as the default (levels 0-4, level 0 from cin 64): GPU suite, smoke,
# fp32 stream bitwise, default bench (parity + CPU baseline), C2.
set -u
O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bitwise_fp32 timeout -k 10 240 python tools/stream_bitwise.py --precision fp32 --height 720 --width 1280 --batch 4 --rounds 3
step bench timeout -k 10 400 python bench.py
step c2 timeout -k 10 200 python bench.py --height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-pairs 1 --no-alt
step c2_graph timeout -k 10 200 python bench.py --height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt --graph
exit 0
