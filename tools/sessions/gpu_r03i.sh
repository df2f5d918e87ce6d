#!/bin/bash
# Round 3: ablations of the cfg 20 Winograd tile (lab bits 1024 + ABL):
# 0 base, 3 no DMA, 4 no MFMA, 8 no transform, 16 no window reads, 32 no U reads,
# 48 no LDS reads, 56 no reads + no transform, 59 + no DMA, 64 no stores, 123 all but MFMA
set -u
O=gpurun_out/r03i; mkdir -p $O; export TMPDIR=/tmp
for shp in "256 256 3 1 20" "64 32 0 1 20" "128 64 1 1 20"; do
  for abl in 0 3 4 8 16 32 48 56 59 64 123; do
    timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 30 --shape $shp --sched $((1024 + abl)) > $O/abl.tmp 2>&1
    rc=$?; grep -v amdgpu.ids $O/abl.tmp | sed "s/^/abl$abl /"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
