#!/bin/bash
# C3 fp16 (1280x736 x 4) after the ring fix-up rework (fp16 K-run structure, KS 4 spill 28 B), x2
set -u
O=gpurun_out/r03ak; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --cpu-baseline off --no-alt > $O/c3_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 5 --warmup 2 --cpu-baseline off --no-alt > $O/prof.log 2>&1 || exit 1
