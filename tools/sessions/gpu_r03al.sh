#!/bin/bash
# same-box A/B: the build before the ring fix-up rework (ab/pre_edge, a git worktree of
# 9fd4482) vs the current one, C3 fp16 1280x736 x 4 and the default fp32 bench, interleaved
set -u
O=$PWD/gpurun_out/r03al; mkdir -p $O; export TMPDIR=/tmp
C3="--height 736 --width 1280 --batch 4 --precision fp16 --cpu-baseline off --no-alt"
for r in 1 2; do
  (cd ab/pre_edge && timeout -k 10 300 python bench.py $C3 > $O/c3_old_$r.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py $C3 > $O/c3_new_$r.log 2>&1 || exit 1
  (cd ab/pre_edge && timeout -k 10 300 python bench.py --cpu-baseline off --no-alt > $O/fp32_old_$r.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py --cpu-baseline off --no-alt > $O/fp32_new_$r.log 2>&1 || exit 1
done
