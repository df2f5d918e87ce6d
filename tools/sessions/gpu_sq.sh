#!/bin/bash
# SQ counters (one --pmc pass, <= 8 SQ + GRBM) over a short bench run
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_bench -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt > gpurun_out/sq_bench.log 2>&1
echo "sq rc=$?"
