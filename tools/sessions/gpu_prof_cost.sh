#!/bin/bash
# Cost of bench.py's per-launch HIP-event profiler on the measured rate:
# default bench with and without --no-prof, interleaved, at 720p x4 and C2.
set -u
mkdir -p gpurun_out
ARGS="--steps 10 --warmup 3 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/pc_prof_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $ARGS --no-prof > gpurun_out/pc_noprof_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $C2 > gpurun_out/pc_c2_prof_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $C2 --no-prof > gpurun_out/pc_c2_noprof_$r.log 2>&1 || exit 1
done
for f in gpurun_out/pc_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
