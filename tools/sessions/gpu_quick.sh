#!/bin/bash
# GPU round trip: full -m gpu suite, then one bench line (stops at the first failure).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -15 gpurun_out/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
tail -1 gpurun_out/bench.log | cut -c1-1500
exit $rc
