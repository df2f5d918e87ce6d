#!/bin/bash
# BASELINE config lines on one GPU: C3 (1280x736 fp16 x4), C5 per-GPU share (4K fp16 x1, split16 x2).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --cpu-baseline off > gpurun_out/bench_c3_fp16_1280x736x4.log 2>&1 && tail -1 gpurun_out/bench_c3_fp16_1280x736x4.log | cut -c1-300 && \
timeout -k 10 400 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --precision fp16 --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_4k_fp16x1.log 2>&1 && tail -1 gpurun_out/bench_4k_fp16x1.log | cut -c1-300 && \
timeout -k 10 400 python bench.py --height 2176 --width 3840 --batch 2 --steps 5 --warmup 2 --cpu-baseline off --no-alt > gpurun_out/bench_4k_split16x2.log 2>&1 && tail -1 gpurun_out/bench_4k_split16x2.log | cut -c1-300
