#!/bin/bash
# Dead-row MFMA skip A/B: A = ab/librrin_hip_prev.so, B = in-tree library.
# GPU parity first (conv / net / config tests), then interleaved benches:
# default (720p x 4, 2 streams, fp32), C2 640x368 x 1 fp32, 720p x 1 fp32,
# default split16; then the fp32 tile sweeps at C2 and 720p x 1.
set -u
mkdir -p gpurun_out/ab
A='import sys, rrin_amd._lib as L; L.LIB_PATH = "ab/librrin_hip_prev.so"; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_net.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?
tail -2 gpurun_out/ab/tests.log; [ $rc -ne 0 ] && exit $rc
C="--steps 10 --warmup 3 --cpu-baseline off --no-alt"
S="--steps 20 --warmup 5 --cpu-baseline off --no-alt --batch 1 --streams 1"
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then P=(python -c "$A"); else P=(python bench.py); fi
    timeout -k 10 300 "${P[@]}" $C > gpurun_out/ab/def_${v}_$r.log 2>&1 || exit 1
    timeout -k 10 300 "${P[@]}" $S --height 368 --width 640 > gpurun_out/ab/c2_${v}_$r.log 2>&1 || exit 1
    timeout -k 10 300 "${P[@]}" $S --height 720 --width 1280 > gpurun_out/ab/p1_${v}_$r.log 2>&1 || exit 1
    timeout -k 10 300 "${P[@]}" $C --precision fp32_split16 > gpurun_out/ab/s16_${v}_$r.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab/*_[12].log; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], r['frac'], 'ms', d['ms_per_step'], 'unprof', d.get('unprofiled',{}).get('value'))"; done
timeout -k 10 500 python tools/conv_lab.py tune --precision fp32 --height 368 --width 640 --batch 1 --reps 7 --out gpurun_out/ab/tune_c2.json > gpurun_out/ab/tune_c2.txt 2>&1 && \
timeout -k 10 500 python tools/conv_lab.py tune --precision fp32 --height 720 --width 1280 --batch 1 --reps 7 --out gpurun_out/ab/tune_720x1.json > gpurun_out/ab/tune_720x1.txt 2>&1
