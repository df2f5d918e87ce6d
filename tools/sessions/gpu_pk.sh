#!/bin/bash
# Packed-FP32 experiment.  Library variants (make pk-variants):
#   pk_all  - packed FP32 VALU ops in every kernel (the round-1 v10 build flags)
#   pk_edge - only the sub-pixel ring fix-up (edge_fix_h8_kernel) packed
#   pk_conv - only the conv kernels (conv3x3_h8_kernel, epilogues) packed
# Each is swapped in for librrin_hip.so and runs the concurrency regression
# (a DMA+MFMA conv looping on a side stream beside 18 forwards) once; a failing
# test is a result here, a fault / timeout ends the script.  Then the default
# bench (no CPU baseline) on the NOPK library and on pk_conv, interleaved.
set -u
mkdir -p gpurun_out/pk
cp rrin_amd/librrin_hip.so gpurun_out/pk/nopk.so.bak
run_conc() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py -v --timeout 240 --timeout-method thread \
    > gpurun_out/pk/conc_$1.log 2>&1
  rc=$?
  echo "variant $1: pytest rc=$rc"; grep -E "PASSED|FAILED|differ" gpurun_out/pk/conc_$1.log | head -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for v in pk_edge pk_conv pk_all; do
  cp rrin_amd/librrin_hip_$v.so rrin_amd/librrin_hip.so
  run_conc $v
done
ARGS="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in 1 2; do
  cp gpurun_out/pk/nopk.so.bak rrin_amd/librrin_hip.so
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/pk/bench_nopk_$r.log 2>&1 || exit 1
  cp rrin_amd/librrin_hip_pk_conv.so rrin_amd/librrin_hip.so
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/pk/bench_pk_conv_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $ARGS --precision fp32_split16 > gpurun_out/pk/bench_s16_pk_conv_$r.log 2>&1 || exit 1
  cp gpurun_out/pk/nopk.so.bak rrin_amd/librrin_hip.so
  timeout -k 10 300 python bench.py $ARGS --precision fp32_split16 > gpurun_out/pk/bench_s16_nopk_$r.log 2>&1 || exit 1
done
cp gpurun_out/pk/nopk.so.bak rrin_amd/librrin_hip.so
rm -f gpurun_out/pk/nopk.so.bak
for f in gpurun_out/pk/bench_*.log; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], 'conv_busy', r.get('conv_busy_ms_per_step'), 'head', r.get('head_ms_per_step'))"; done
