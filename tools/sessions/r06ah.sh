#!/bin/bash
# Round 6 call ah: C2 kernel families (rocprofv3 kernel stats) on the final build.
set -u
O=gpurun_out/r06ah; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --height 368 --width 640 --batch 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt > $O/prof.log 2>&1 || exit $?
head -14 $O/prof/run_kernel_stats.csv | cut -d, -f1-6
exit 0
