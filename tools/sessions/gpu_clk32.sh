#!/bin/bash
# effective clock + MFMA busy of fp32 conv ablation variants (one --pmc pass each)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "128 64 1 1 4 0" "128 64 1 1 4 1" "128 64 1 1 4 13" "256 256 3 1 4 0" "256 256 3 1 4 1" "256 256 3 1 4 13"; do
  set -- $spec
  tag=clk32_$1_$2_$3_$5_x$6
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/$tag -o run -- python3 tools/conv_lab.py single --precision fp32_planar --batch 2 --reps 40 --shape $1 $2 $3 $4 $5 --sched $6 > gpurun_out/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; grep fp32_planar: gpurun_out/$tag.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/$tag.log; exit $rc; fi
done
