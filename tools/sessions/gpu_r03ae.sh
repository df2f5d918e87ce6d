#!/bin/bash
# forward-part streams at 1280x720 x 4 (default 2), interleaved
set -u
O=gpurun_out/r03ae; mkdir -p $O; export TMPDIR=/tmp
ARGS="--cpu-baseline off --no-alt"
for r in 1 2; do
  for s in 2 3 4 1; do
    timeout -k 10 200 python bench.py $ARGS --streams $s > $O/s${s}_$r.log 2>&1 || exit 1
  done
  timeout -k 10 200 python bench.py $ARGS --batch 8 --streams 2 > $O/b8s2_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $ARGS --batch 8 --streams 4 > $O/b8s4_$r.log 2>&1 || exit 1
done
