#!/bin/bash
# RCCL path at world size 1 (bench --dist-init, nccl), then the C5 (4K) tile sweeps
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run bench_nccl1 300 python bench.py --steps 5 --warmup 2 --dist-init --dist-backend nccl --cpu-baseline off --no-alt
run tune4k_fp16 600 python tools/conv_lab.py tune --precision fp16 --batch 1 --height 2176 --width 3840 --reps 3 --out gpurun_out/tune4k_fp16.json
run tune4k_fp32 600 python tools/conv_lab.py tune --precision fp32 --batch 1 --height 2176 --width 3840 --reps 3 --out gpurun_out/tune4k_fp32.json
run bench4k_fp16 300 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --steps 5 --warmup 2 --precision fp16 --cpu-baseline off --no-alt
run bench4k_fp32 300 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --steps 3 --warmup 1 --precision fp32 --cpu-baseline off --no-alt
