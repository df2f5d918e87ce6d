#!/bin/bash
# Winograd instruction-order variants (lab bits 16 / 32) vs the base schedule:
# record-conv parity first, then interleaved single-conv timings (librrin_lab.so).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "${NOTEST:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h8.log 2>&1
rc=$?; echo "tests_h8 rc=$rc"; tail -3 gpurun_out/tests_h8.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for shp in "256 256 3 1 18" "64 32 0 1 18" "128 64 1 1 18" "512 512 4 1 18"; do
  for abl in ${ABLS:-0 64 128 32}; do
    timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 40 --shape $shp --sched $abl > gpurun_out/abl.tmp 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/abl.tmp | sed "s/^/r$rep abl$abl /"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
done
exit 0
