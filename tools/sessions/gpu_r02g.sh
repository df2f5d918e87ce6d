#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python tools/conv_lab.py tune --precision fp32 --batch 4 --reps 3 --out gpurun_out/tune32r_b4.json > gpurun_out/tune32r_b4.log 2>&1
echo rc=$?; tail -3 gpurun_out/tune32r_b4.log | cut -c1-200
