#!/bin/bash
# Round 4 session k: kernel trace of the C2 forward (one stream) to price the launch
# gaps between kernels (graph-capture candidate).
set -u
O=${O:-gpurun_out/r04k}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt --no-prof > $O/prof_c2.log 2>&1
echo "rc=$?"; tail -2 $O/prof_c2.log | cut -c1-300
