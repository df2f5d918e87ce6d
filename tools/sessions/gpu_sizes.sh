#!/bin/bash
# GPU tests + bench lines at the three tile-table size classes (C2 640x368 x1,
# 720p x1, default 720p x4) with the size-class tile tables.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 && tail -2 gpurun_out/tests.log && \
timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_640x368x1.log 2>&1 && tail -1 gpurun_out/bench_c2_640x368x1.log | cut -c1-400 && \
timeout -k 10 300 python bench.py --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt > gpurun_out/bench_1280x720x1.log 2>&1 && tail -1 gpurun_out/bench_1280x720x1.log | cut -c1-400 && \
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log | cut -c1-400 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 10 --warmup 3 --cpu-baseline off --no-alt > gpurun_out/prof_c2.log 2>&1
