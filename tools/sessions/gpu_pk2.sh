#!/bin/bash
# Packed-FP32 experiment, part 2: the ring fix-up's FMAs as
# hand-placed v_pk_fma_f32 (everything else unpacked) - pk_asm1 splat src1 pair,
# no op_sel; pk_asm2 the compiler's op_sel:[0,1,0] form - and the NOPK library,
# each through the fp16 concurrency regression with 24 rounds (72 forwards).
set -u
mkdir -p gpurun_out/pk
cp rrin_amd/librrin_hip.so gpurun_out/pk/nopk.so.bak
for v in pk_asm1 pk_asm2 nopk; do
  if [ $v = nopk ]; then cp gpurun_out/pk/nopk.so.bak rrin_amd/librrin_hip.so; else cp rrin_amd/librrin_hip_$v.so rrin_amd/librrin_hip.so; fi
  RRIN_CONC_ROUNDS=24 timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py -k "fp16 or split16" -v \
    --timeout 240 --timeout-method thread > gpurun_out/pk/conc24_$v.log 2>&1
  rc=$?
  echo "variant $v: pytest rc=$rc"; grep -E "PASSED|FAILED|differ" gpurun_out/pk/conc24_$v.log | head -8
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
cp gpurun_out/pk/nopk.so.bak rrin_amd/librrin_hip.so && rm -f gpurun_out/pk/nopk.so.bak
