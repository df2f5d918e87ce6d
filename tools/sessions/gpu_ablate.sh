#!/bin/bash
# kernel lab: schedule variants / ablations of the split16 conv (librrin_lab.so)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/conv_lab.py ablate --reps ${REPS:-7} --out gpurun_out/ablate.json > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; cut -c1-900 gpurun_out/ablate.log
exit $rc
