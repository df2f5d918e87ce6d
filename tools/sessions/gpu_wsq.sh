#!/bin/bash
# Winograd kernel counters (SQ waits / MFMA busy / LDS conflicts) on three conv shapes,
# then config sweeps (tail_finite first convs) at 720p x 2 and at the C2 size 640x368 x 1.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for shp in "256 256 3 1 18" "64 32 0 1 18" "32 32 0 1 18" "256 256 3 1 3"; do
  tag=$(echo $shp | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_$tag -o run -- python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 20 --shape $shp > gpurun_out/sq_$tag.log 2>&1
  rc=$?; echo "sq $tag rc=$rc"; tail -2 gpurun_out/sq_$tag.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -u tools/conv_lab.py tune --precision fp32 --batch 2 --reps 7 --out gpurun_out/tune_x2.json > gpurun_out/tune_x2.log 2>&1
echo "tune x2 rc=$?"
timeout -k 10 600 python -u tools/conv_lab.py tune --precision fp32 --batch 1 --height 368 --width 640 --reps 7 --out gpurun_out/tune_c2.json > gpurun_out/tune_c2.log 2>&1
echo "tune c2 rc=$?"
exit 0
