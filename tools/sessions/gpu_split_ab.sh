#!/bin/bash
# uneven / more-stream batch splits of the default bench (unprofiled), interleaved
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-alt --no-prof "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1:], d['value'])" "$@"; }
for i in 1 2; do
run --streams 2 || exit 1
run --split 1,3 || exit 1
run --split 3,1 || exit 1
run --streams 3 || exit 1
run --streams 4 || exit 1
done
