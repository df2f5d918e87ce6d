#!/bin/bash
# C2 (640x368 x 1, one stream) kernel trace: per-launch durations and the gaps between
# consecutive launches (--no-prof: no HIP events between the kernels)
set -u
O=gpurun_out/r03af; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-prof --no-alt > $O/c2.log 2>&1 || exit 1
f=$(ls $O/prof/*/run_kernel_trace.csv 2>/dev/null || ls $O/prof/run_kernel_trace.csv); ls -la $O/prof
gzip -c $f > $O/c2_kernel_trace.csv.gz
