#!/bin/bash
# h8 conv parity (every tile config) + per-shape config sweep of the split16 / fp16 convs
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h8.log 2>&1
rc=$?; echo "tests_h8 rc=$rc"; tail -3 gpurun_out/tests_h8.log
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in ${TUNEPREC:-fp32_split16}; do
  timeout -k 10 600 python -u tools/conv_lab.py tune --precision $prec --out gpurun_out/tune_$prec.json > gpurun_out/tune_$prec.log 2>&1
  rc=$?; echo "tune $prec rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
