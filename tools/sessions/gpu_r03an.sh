#!/bin/bash
# same-box A/B: pre-rework build vs current (fp16 fix-up: no preload, compile-time single run, plain loop); C3 x3 and fp32 default x2
set -u
O=$PWD/gpurun_out/r03an; mkdir -p $O; export TMPDIR=/tmp
C3="--height 736 --width 1280 --batch 4 --precision fp16 --cpu-baseline off --no-alt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_h8.py -m gpu -x -q -k "subpixel or edge" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  (cd ab/pre_edge && timeout -k 10 300 python bench.py $C3 > $O/c3_old_$r.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py $C3 > $O/c3_new_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  (cd ab/pre_edge && timeout -k 10 300 python bench.py --cpu-baseline off --no-alt > $O/fp32_old_$r.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py --cpu-baseline off --no-alt > $O/fp32_new_$r.log 2>&1 || exit 1
done
