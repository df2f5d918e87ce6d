#!/bin/bash
# device-cached t coefficients (engine.COEF_CACHE) A/B, interleaved
set -u
O=gpurun_out/r03ad; mkdir -p $O; export TMPDIR=/tmp
B='import sys, rrin_amd.engine as E; E.RRINEngine.COEF_CACHE = False; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
ARGS="--cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py $ARGS > $O/c1_cache_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -c "$B" $ARGS > $O/c1_nocache_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $C2 > $O/c2_cache_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -c "$B" $C2 > $O/c2_nocache_$r.log 2>&1 || exit 1
done
tail -1 $O/tests.log
