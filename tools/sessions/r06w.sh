#!/bin/bash
# Round 6 call w: kind 6 (exact fp32 and fp16) with zero-C first MFMAs: its tests, the training
# line (kinds 6 / 7 forward and dgrad), C3.
set -u
O=gpurun_out/r06w; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run tk6 400 python -u -m pytest tests/test_gpu_winoh.py tests/test_gpu_train.py tests/test_gpu_split.py -m gpu -x -q --timeout 120 --timeout-method thread
run train 300 python bench.py --train --steps 5 --warmup 2
run c3 200 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt
exit 0
