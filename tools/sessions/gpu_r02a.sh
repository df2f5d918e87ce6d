#!/bin/bash
# round 2 baseline: GPU tests, exact-fp32 bench, fp32 breakdown / sweep at the 2-pair part size
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench32 300 python bench.py --steps 10 --warmup 3 --precision fp32 --cpu-baseline off
run brk32 300 python tools/conv_lab.py breakdown --precision fp32 --batch 2 --out gpurun_out/brk32.json
run tune32 400 python tools/conv_lab.py tune --precision fp32 --batch 2 --out gpurun_out/tune32.json
