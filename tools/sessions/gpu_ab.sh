#!/bin/bash
# A/B of tile tables in the default bench (unprofiled; interleaved rounds)
# usage: A='{json}' B='{json}' bash tools/sessions/gpu_ab.sh
mkdir -p gpurun_out
A=${A:-'{}'}
run() { timeout -k 10 300 python tools/bench_ab.py "$1" -- --steps 10 --warmup 3 --cpu-baseline off --no-alt --no-prof 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['value'])" "$1"; }
for i in 1 2 3; do
run "$A" || exit 1
run "$B" || exit 1
[ -n "${C:-}" ] && { run "$C" || exit 1; }
done
exit 0
