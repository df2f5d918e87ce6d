#!/bin/bash
# SQ counters of single exact-fp32 conv shapes (one --pmc pass each, <= 8 SQ + GRBM)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "128 64 1 1 4 0" "64 32 0 1 3 1" "512 512 4 1 4 0" "32 32 0 1 0 0"; do
  set -- $spec
  tag=sq32_$1_$2_$3_$5_s$6
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$tag -o run -- python3 tools/conv_lab.py single --precision fp32_planar --batch 2 --reps 20 --shape $1 $2 $3 $4 $5 --src $6 > gpurun_out/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/$tag.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
