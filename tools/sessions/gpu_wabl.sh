#!/bin/bash
# Winograd kernel: record-conv parity, then lab ablation bits (librrin_lab.so, --sched): 0 base,
# 1 no weight DMA, 2 no raw DMA, 3 no DMA, 4 no MFMA, 8 no transform arithmetic, 11, 15 combined
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h8.log 2>&1
rc=$?; echo "tests_h8 rc=$rc"; tail -3 gpurun_out/tests_h8.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
for shp in "256 256 3 1 18" "64 32 0 1 18" "128 64 1 1 18"; do
  for abl in ${ABLS:-0 3 4 8 11}; do
    timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 30 --shape $shp --sched $abl > gpurun_out/abl.tmp 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/abl.tmp | sed "s/^/abl$abl /"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
