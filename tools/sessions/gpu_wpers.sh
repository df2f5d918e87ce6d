#!/bin/bash
# Persistent Winograd grid (lab bit 256) vs one tile per block: bitwise check
# against the product kernel per shape, then interleaved single-conv timings.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for shp in "256 256 3 1 18" "64 32 0 1 18" "32 32 0 1 18" "16 32 0 1 18" "128 64 1 1 18" "512 512 4 1 18" "64 64 1 1 18"; do
  timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 3 --shape $shp --sched 256 --check > gpurun_out/chk.tmp 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/chk.tmp | grep check
  if [ $rc -ne 0 ]; then cat gpurun_out/chk.tmp; exit $rc; fi
done
for rep in 1 2; do
for shp in "256 256 3 1 18" "64 32 0 1 18" "32 32 0 1 18" "16 32 0 1 18" "128 64 1 1 18" "512 512 4 1 18" "64 64 1 1 18"; do
  for abl in ${ABLS:-0 256}; do
    timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 40 --shape $shp --sched $abl > gpurun_out/abl.tmp 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/abl.tmp | sed "s/^/r$rep abl$abl /"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
done
exit 0
