#!/bin/bash
# A/B of two builds of librrin_hip.so in one box session: A = ab/librrin_hip_prev.so
# (the previous build), B = the in-tree library; interleaved A B A B, default bench.
set -u
mkdir -p gpurun_out
ARGS="--steps 10 --warmup 3 --cpu-baseline off --no-alt"
A='import sys, rrin_amd._lib as L; L.LIB_PATH = "ab/librrin_hip_prev.so"; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 && tail -1 gpurun_out/tests.log || exit 1
for r in 1 2; do
  timeout -k 10 300 python -c "$A" $ARGS > gpurun_out/ab_prev_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_new_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python -c "$A" --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt > gpurun_out/ab_c2_prev_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt > gpurun_out/ab_c2_new_$r.log 2>&1 || exit 1
done
for f in gpurun_out/ab_*.log; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], 'head_ms', r['head_ms_per_step'], 'conv_busy', r['conv_busy_ms_per_step'])"; done
