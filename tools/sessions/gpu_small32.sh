#!/bin/bash
# Exact fp32 at the small / batch-1 workloads with the small / medium tables:
# size-class parity tests, then C2 640x368 x 1 and 720p x 1 benches.
set -u
mkdir -p gpurun_out/s32
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -m gpu -x -q -k "size_class or golden" --timeout 300 --timeout-method thread > gpurun_out/s32/tests.log 2>&1; rc=$?
tail -2 gpurun_out/s32/tests.log; [ $rc -ne 0 ] && exit $rc
S="--steps 20 --warmup 5 --cpu-baseline off --no-alt --batch 1 --streams 1"
timeout -k 10 300 python bench.py $S --height 368 --width 640 > gpurun_out/s32/c2_fp32.log 2>&1 && \
timeout -k 10 300 python bench.py $S --height 720 --width 1280 > gpurun_out/s32/p1_fp32.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --height 368 --width 640 --batch 1 --streams 1 > gpurun_out/s32/c2_fp32_full.log 2>&1
rc=$?
for f in gpurun_out/s32/*.log; do [ -s $f ] && python -c "
import json
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
    print('$f', d['value'], r['frac'], 'ms', d['ms_per_step'], 'unprof', d.get('unprofiled',{}).get('value'), 'ring', r.get('subpixel_ring_fix_ms_per_step'), 'head', r.get('head_ms_per_step'))
except Exception: pass"; done
exit $rc
