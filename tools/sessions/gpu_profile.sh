#!/bin/bash
# rocprofv3 kernel stats of the default bench + PMC HBM traffic passes (separate
# FETCH_SIZE / WRITE_SIZE runs) + fp16 bench lines of the BASELINE fp16 configs
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=prof,pmc PMCPREC="${PMCPREC:-fp32_split16 fp16}" bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --precision fp16 --height 736 --batch 4 --cpu-baseline off --no-alt > gpurun_out/bench_fp16_736x4.log 2>&1; echo "fp16 736 rc=$?"
exit 0
