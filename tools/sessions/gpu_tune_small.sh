#!/bin/bash
# Parity of every tile config, then the per-shape tile sweep at the small /
# batch-1 workloads (C2 640x368x1, 720p x1) for the engine's size-class tables.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h8.log 2>&1 && tail -1 gpurun_out/tests_h8.log && \
timeout -k 10 400 python tools/conv_lab.py tune --precision fp32_split16 --height 368 --width 640 --batch 1 --reps 7 --out gpurun_out/tune_c2.json > gpurun_out/tune_c2.txt 2>&1 && \
timeout -k 10 400 python tools/conv_lab.py tune --precision fp32_split16 --height 720 --width 1280 --batch 1 --reps 7 --out gpurun_out/tune_720x1.json > gpurun_out/tune_720x1.txt 2>&1
