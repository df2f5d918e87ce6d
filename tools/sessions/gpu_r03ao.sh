#!/bin/bash
# A/B: ring fix-up cross split up to 512 workgroups (ab/librrin_hip_x512.so) vs 256 (in tree), default bench, interleaved x3
set -u
O=gpurun_out/r03ao; mkdir -p $O; export TMPDIR=/tmp
ARGS="--cpu-baseline off --no-alt"
A='import sys, rrin_amd._lib as L; L.LIB_PATH = "ab/librrin_hip_x512.so"; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $ARGS > $O/x256_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -c "$A" $ARGS > $O/x512_$r.log 2>&1 || exit 1
done
