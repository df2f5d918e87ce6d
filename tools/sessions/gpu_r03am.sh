#!/bin/bash
# same-box A/B, C3 fp16 1280x736 x 4: pre-rework build (ab/pre_edge) vs the current one with the plain fp16 fix-up loop
set -u
O=$PWD/gpurun_out/r03am; mkdir -p $O; export TMPDIR=/tmp
C3="--height 736 --width 1280 --batch 4 --precision fp16 --cpu-baseline off --no-alt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_h8.py -m gpu -x -q -k "subpixel or edge" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  (cd ab/pre_edge && timeout -k 10 300 python bench.py $C3 > $O/c3_old_$r.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py $C3 > $O/c3_new_$r.log 2>&1 || exit 1
done
