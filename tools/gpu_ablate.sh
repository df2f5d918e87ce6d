#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_net.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h8net.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests_h8net.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "=== ablate"
timeout -k 10 500 python -u tools/conv_lab.py ablate --reps 7 --out gpurun_out/ablate.json > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; cat gpurun_out/ablate.log | cut -c1-600
exit 0
