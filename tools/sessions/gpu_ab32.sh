#!/bin/bash
# exact-fp32 conv ablations (librrin_lab32.so) at the 2-pair part size
set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_lab.py ablate32 --batch 2 --reps 7 --out gpurun_out/ablate32.json > gpurun_out/ablate32.log 2>&1
rc=$?; echo "ablate32 rc=$rc"; cat gpurun_out/ablate32.log; exit $rc
