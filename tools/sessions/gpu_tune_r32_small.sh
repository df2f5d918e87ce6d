#!/bin/bash
# Exact-fp32 (R32) at the small / batch-1 workloads: C2 bench before tuning,
# then the per-shape tile sweeps for the engine's small / medium tables.
set -u
mkdir -p gpurun_out/r32s
B="--steps 20 --warmup 5 --cpu-baseline off --no-alt --batch 1 --streams 1"
timeout -k 10 300 python bench.py $B --height 368 --width 640 > gpurun_out/r32s/bench_c2_fp32_pre.log 2>&1 && \
timeout -k 10 300 python bench.py $B --height 368 --width 640 --precision fp32_planar > gpurun_out/r32s/bench_c2_fp32planar.log 2>&1 && \
timeout -k 10 300 python bench.py $B --height 720 --width 1280 > gpurun_out/r32s/bench_720x1_fp32_pre.log 2>&1 && \
timeout -k 10 500 python tools/conv_lab.py tune --precision fp32 --height 368 --width 640 --batch 1 --reps 7 --out gpurun_out/r32s/tune_c2.json > gpurun_out/r32s/tune_c2.txt 2>&1 && \
timeout -k 10 500 python tools/conv_lab.py tune --precision fp32 --height 720 --width 1280 --batch 1 --reps 7 --out gpurun_out/r32s/tune_720x1.json > gpurun_out/r32s/tune_720x1.txt 2>&1
rc=$?
for f in gpurun_out/r32s/bench_*.log; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], r['frac'], 'ring', r.get('subpixel_ring_fix_ms_per_step'), 'head', r.get('head_ms_per_step'), 'ms', d['ms_per_step'])"; done
exit $rc
