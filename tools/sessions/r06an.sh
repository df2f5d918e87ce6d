#!/bin/bash
# Round 6 call an: the persistent short-K kind 14 under concurrency -- the side-stream bitwise
# test (persistent case) and repeated whole forwards at the headline size, 1 vs 2 streams bitwise.
set -u
O=gpurun_out/r06an; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -6 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run side 300 python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q -k "side_stream" --timeout 200 --timeout-method thread
run sbw 400 python tools/stream_bitwise.py --precision fp32 --height 720 --width 1280 --batch 4 --rounds 6
exit 0
