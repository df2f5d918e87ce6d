#!/bin/bash
# Winograd F(2x2,3x3) exact-fp32 config: record-conv parity (every config, incl. Winograd),
# then the per-shape sweep of every F32R config at 1280x720 x 2 pairs (the 2-stream part size).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread ${PYK:-} > gpurun_out/tests_h8.log 2>&1
rc=$?; echo "tests_h8 rc=$rc"; tail -15 gpurun_out/tests_h8.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/conv_lab.py tune --precision fp32 --batch ${TBATCH:-2} --reps 7 --out gpurun_out/tune_wino.json > gpurun_out/tune_wino.log 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/tune_wino.log | cut -c1-200
exit $rc
