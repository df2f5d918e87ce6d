#!/bin/bash
# F(4x4) kernel (cfg 22) ablations (librrin_lab.so): 0 base, 1 no DMA, 3 no DMA/wait/barrier,
# 4 no MFMA, 8 no transform, 12 neither, 32 no U reads, 35, 43; cfg 20 base for reference
set -u
O=gpurun_out/r03p; mkdir -p $O; export TMPDIR=/tmp
for shp in "256 128 2 1 22" "64 32 0 1 22"; do
  for abl in 0 1 3 4 8 12 32 35 43; do
    timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 30 --shape $shp --sched $abl > $O/abl.tmp 2>&1
    rc=$?; grep -v amdgpu.ids $O/abl.tmp | sed "s/^/abl$abl /" | tee -a $O/abl.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for shp in "256 128 2 1 20" "64 32 0 1 20"; do
  timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 30 --shape $shp --sched 1024 > $O/abl.tmp 2>&1
  grep -v amdgpu.ids $O/abl.tmp | sed "s/^/cfg20 /" | tee -a $O/abl.log
done
exit 0
