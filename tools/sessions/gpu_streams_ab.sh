#!/bin/bash
# streams / batch A/B of the default bench (profiled and unprofiled), interleaved
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-alt "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(sys.argv[1:], d['value'], r.get('conv_ms_per_step'), r.get('head_ms_per_step'))" "$@"; }
for i in 1 2; do
run || exit 1
run --streams 2 || exit 1
run --no-prof || exit 1
run --no-prof --streams 2 || exit 1
run --no-prof --streams 2 --batch 8 || exit 1
done
